"""Multi-task evaluation protocol on the GPU simulator (evaluation.py:13-98).

`EvaluationProtocol` keeps the reference's contract: a subclass names a `run_id` and implements
`obtain_scores(env_name)` returning at least `n_rollouts` eval scores; `do_eval()` evaluates the demo
env and every test variant of it (`DEMO_ENVS_TO_TEST_ENVS_MAP`) and returns one record per test env
with the mean score, the two-sided 95% t confidence interval of the mean and the sample std
(ddof=1), truncating extra scores with a warning as the reference does.  The reference computes the
interval with statsmodels' `DescrStatsW(scores).tconfint_mean(0.05)`; statsmodels is absent here, so
`tconfint_mean` restates it (mean +- t_{0.975, n-1} * std / sqrt(n)) with scipy's t quantile.

`BatchedEvaluationProtocol` is the GPU-native subclass: the `n_rollouts` episodes of each env run as
one batch of envs on one MI355X (`make_vec`, one episode per env, no auto-reset), driven by a
policy callable mapping the observation dict of device tensors to uint8 actions.
"""
import abc
import collections
import warnings

import numpy as np
import torch

from . import make_vec, registry


def tconfint_mean(scores, alpha=0.05):
    """statsmodels DescrStatsW(scores).tconfint_mean(alpha, 'two-sided') (unweighted)."""
    from scipy import stats
    x = np.asarray(scores, dtype=np.float64)
    n = len(x)
    mean = x.mean()
    std_mean = x.std(ddof=1) / np.sqrt(n)
    q = stats.t.ppf(1 - alpha / 2.0, n - 1)
    return mean - q * std_mean, mean + q * std_mean


class EvaluationProtocol(abc.ABC):
    """evaluation.py:13-98"""
    _called_init = False

    def __init__(self, demo_env_name, n_rollouts):
        self.n_rollouts = n_rollouts
        self.demo_env_name = demo_env_name
        self.test_env_names = [demo_env_name, *registry.DEMO_ENVS_TO_TEST_ENVS_MAP[demo_env_name]]
        self._called_init = True

    @property
    @abc.abstractmethod
    def run_id(self):
        """Identifier of the evaluated model / algorithm (the `run_id` column)."""

    @abc.abstractmethod
    def obtain_scores(self, env_name):
        """At least `self.n_rollouts` eval scores of rollouts on `env_name`."""

    def do_eval(self, verbose=False):
        if not self._called_init:
            raise ValueError("EvaluationProtocol.__init__() was not called. Did you include a "
                             "super().__init__(...) call in your subclass?")
        records = []
        for env_name in self.test_env_names:
            scores = list(self.obtain_scores(env_name))
            if len(scores) < self.n_rollouts:
                raise ValueError(f".obtain_scores() returned only {len(scores)} scores, but we asked for "
                                 f"{self.n_rollouts} scores")
            if len(scores) > self.n_rollouts:
                warnings.warn(f"Asked for {self.n_rollouts} scores but got {len(scores)} scores instead. "
                              f"Will truncate to only consider the first {self.n_rollouts} scores.")
                scores = scores[:self.n_rollouts]
            lo, hi = tconfint_mean(scores)
            records.append(collections.OrderedDict([
                ("demo_env", self.demo_env_name), ("test_env", env_name), ("mean_score", float(np.mean(scores))),
                ("ci95_lower", float(lo)), ("ci95_upper", float(hi)), ("std_score", float(np.std(scores, ddof=1))),
                ("run_id", self.run_id)]))
        try:
            import pandas as pd
            frame = pd.DataFrame.from_records(records)
        except ImportError:  # pragma: no cover - pandas is present in this image
            frame = records
        if verbose:
            print(f"Final mean scores for '{self.run_id}':")
            for r in records:
                print(f"  {r['test_env']:45s} {r['mean_score']:.3f} [{r['ci95_lower']:.3f}, {r['ci95_upper']:.3f}]")
        return frame


class BatchedEvaluationProtocol(EvaluationProtocol):
    """n_rollouts episodes of each env in one GPU batch; policy(obs_dict) -> uint8 actions [N]."""

    def __init__(self, demo_env_name, n_rollouts, policy, run_id="policy", device="cuda:0", base_seed=0):
        super().__init__(demo_env_name, n_rollouts)
        self.policy = policy
        self._run_id = run_id
        self.device = device
        self.base_seed = base_seed

    @property
    def run_id(self):
        return self._run_id

    def obtain_scores(self, env_name):
        n = self.n_rollouts
        vec = make_vec(env_name, n, device=self.device, seeds=[self.base_seed + i for i in range(n)], auto_reset=False)
        try:
            obs = vec.reset()
            scores = None
            for _ in range(vec.max_episode_steps):
                obs, _, done, info = vec.step(self.policy(obs))
                if bool(done.all()):
                    scores = info["eval_score"].cpu().numpy().copy()
                    break
            if scores is None:
                raise RuntimeError(f"{env_name}: episodes did not end after {vec.max_episode_steps} steps")
            return scores.tolist()
        finally:
            vec.close()


def random_policy(num_envs, device="cuda:0", seed=0):
    """Uniform random actions over Discrete(18), like action_space.sample() (device tensors)."""
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    return lambda obs: torch.randint(0, 18, (num_envs,), generator=gen, device=device, dtype=torch.int64).to(torch.uint8)


def latexify_results(eval_data, id_column="run_id"):
    """evaluation.py:101-154: a LaTeX table of a `do_eval()` frame (or of several runs' frames
    concatenated): one column per test env (in order of first appearance), one row per value of
    `id_column`, cells "mean ($\\pm$ std)" with two decimals.  Same text as the reference, including its
    layout quirk of closing the tabular after every algorithm row; a (run, env) pair that is not exactly
    one record raises ValueError with the reference's message."""
    rows = eval_data.to_dict("records") if hasattr(eval_data, "to_dict") else list(eval_data)

    def unique(key):
        seen = []
        for r in rows:
            if r[key] not in seen:
                seen.append(r[key])
        return seen

    test_envs, alg_names = unique("test_env"), unique(id_column)
    col_names = [r"\textbf{%s}" % e for e in test_envs]
    out = [r"\centering" + "\n", r"\begin{tabular}{l@{\hspace{1em}}%s}" % ("c" * len(col_names)) + "\n",
           r"\toprule" + "\n", r"\textbf{Randomisation} & " + " & ".join(col_names) + "\\\\\n", r"\midrule" + "\n"]
    for alg_name in alg_names:
        stat_parts = []
        for env_name in test_envs:
            match = [r for r in rows if r[id_column] == alg_name and r["test_env"] == env_name]
            if len(match) != 1:
                raise ValueError(f"got {len(match)} rows corresponding to {id_column}={alg_name} and "
                                 f"test_env={env_name}, but expected one (maybe IDs in column {id_column} "
                                 f"aren't unique?)")
            row = match[0]
            stat_parts.append(f'{row["mean_score"]:.2f} ($\\pm$ {row["std_score"]:.2f})')
        out.append(r"\textbf{%s} & " % alg_name + " & ".join(stat_parts) + "\\\\\n")
        out.append(r"\bottomrule" + "\n")
        out.append(r"\end{tabular}" + "\n")
    return "".join(out)
