"""Outer training loop (API + loop invariant of src/runs/train/ma_experiment.py:22-283).

Per iteration exactly one ``stepper.run()`` (B episodes, one fused rollout launch) and at most one
``learner.train()`` on ``batch_size`` sampled episodes -- the loop shape that defines the metric.
"""
from __future__ import annotations

import os
import pprint
import time
from types import SimpleNamespace

import torch

from ..components.replay_buffer import ReplayBuffer
from ..components.transforms import OneHot
from ..controllers import REGISTRY as mac_REGISTRY
from ..learners import REGISTRY as learner_REGISTRY
from ..steppers import build_stepper


class LazyTEnv:
    """t_env for a learner's log check without a host sync: call() = the exact value (waits for the runs in
    flight), upper() = an upper bound that needs no wait (the learner skips resolving when even the bound is
    below its next log time)."""

    def __init__(self, stepper):
        self._st = stepper

    def __call__(self) -> int:
        return self._st.t_env

    def upper(self) -> int:
        b = getattr(self._st, "t_env_bounds", None)
        return b()[1] if b is not None else self._st.t_env


def find_latest_model_path(path: str, load_step: int = 0):
    """src/utils/run_utils.py:20-37."""
    steps = [int(n) for n in os.listdir(path) if os.path.isdir(os.path.join(path, n)) and n.isdigit()]
    step = max(steps) if load_step == 0 else min(steps, key=lambda x: abs(x - load_step))
    return os.path.join(path, str(step)), step


class MultiAgentExperiment:
    def __init__(self, args, logger, on_episode_end=None, log_start_t=0):
        self.args = args
        self.logger = logger
        self.on_episode_end = on_episode_end
        self.last_test_T = -self.args.test_interval - 1
        self.last_log_T = 0
        self.model_save_time = 0
        self.learners = []
        self.start_time = time.time()
        self._play_time = None
        self.stepper = self._build_stepper(log_start_t)
        self.env_info = self.stepper.get_env_info()
        env_scheme = self._integrate_env_info()
        if hasattr(self.logger, "update_scheme"):
            self.logger.update_scheme(env_scheme)
        self.groups, self.preprocess, self.scheme = self._build_schemes()
        self._build_learners()
        for learner in self.learners:
            learner.build_optimizer()

    def _build_stepper(self, log_start_t=0):
        return build_stepper(self.args, self.logger, log_start_t)

    def _update_args(self, update):
        self.args = SimpleNamespace(**{**vars(self.args), **update})

    def _integrate_env_info(self):
        env_scheme = {"n_agents": int(self.env_info["n_agents"]), "n_actions": int(self.env_info["n_actions"]),
                      "state_shape": int(self.env_info["state_shape"])}
        if getattr(self.args, "entity_scheme", False):
            env_scheme.update(n_entities=int(self.env_info["n_entities"]),
                              entity_shape=int(self.env_info["entity_shape"]))
        self._update_args(env_scheme)
        self.stepper.args = self.args
        return env_scheme

    def _build_schemes(self):
        if getattr(self.args, "entity_scheme", False):  # REFIL entity scheme (refil_learner.py:81-100)
            NE, ED = self.env_info["n_entities"], self.env_info["entity_shape"]
            scheme = {
                "entities": {"vshape": (NE, ED)},
                "obs_mask": {"vshape": (NE, NE), "dtype": torch.uint8},
                "entity_mask": {"vshape": (NE,), "dtype": torch.uint8},
                "actions": {"vshape": (1,), "group": "agents", "dtype": torch.long},
                "avail_actions": {"vshape": (self.env_info["n_actions"],), "group": "agents", "dtype": torch.int},
                "reward": {"vshape": (1,)},
                "terminated": {"vshape": (1,), "dtype": torch.uint8},
            }
            groups = {"agents": self.args.n_agents}
            preprocess = {"actions": ("actions_onehot", [OneHot(out_dim=self.args.n_actions)])}
            return groups, preprocess, scheme
        scheme = {
            "state": {"vshape": self.env_info["state_shape"]},
            "obs": {"vshape": self.env_info["obs_shape"], "group": "agents"},
            "actions": {"vshape": (1,), "group": "agents", "dtype": torch.long},
            "avail_actions": {"vshape": (self.env_info["n_actions"],), "group": "agents", "dtype": torch.int},
            "reward": {"vshape": (1,)},
            "terminated": {"vshape": (1,), "dtype": torch.uint8},
        }
        groups = {"agents": self.args.n_agents}
        preprocess = {"actions": ("actions_onehot", [OneHot(out_dim=self.args.n_actions)])}
        return groups, preprocess, scheme

    def _build_learners(self):
        a = self.args
        self.home_buffer = ReplayBuffer(self.scheme, self.groups, a.buffer_size, self.env_info["episode_limit"] + 1,
                                        preprocess=self.preprocess,
                                        device="cpu" if a.buffer_cpu_only else a.device)
        self.home_mac = mac_REGISTRY[a.mac](scheme=self.home_buffer.scheme, groups=self.groups, args=a)
        self.home_learner = learner_REGISTRY[a.learner](mac=self.home_mac, scheme=self.home_buffer.scheme,
                                                        logger=self.logger, args=a, name="home")
        self.learners.append(self.home_learner)

    def _init_stepper(self):
        if not self.stepper.is_initalized:
            self.stepper.initialize(scheme=self.scheme, groups=self.groups, preprocess=self.preprocess,
                                    home_mac=self.home_mac)
            # zero-copy insert: train-mode rollouts write straight into the HBM replay ring
            if getattr(self.args, "zero_copy_insert", True) and hasattr(self.stepper, "attach_replay"):
                self.stepper.attach_replay(self.home_buffer)

    def _t_env_reached(self, threshold) -> bool:
        """t_env >= threshold. The interval checks of the loop (t_max, test, save, log) resolve the runs in flight
        only when the bounds of t_env straddle the threshold, so the host keeps running ahead of the device; the
        answer is always the one the exact t_env gives."""
        bounds = getattr(self.stepper, "t_env_bounds", None)
        if bounds is not None:
            lo, hi = bounds()
            if hi < threshold:
                return False
            if lo >= threshold:
                return True
        return self.stepper.t_env >= threshold

    @property
    def _has_not_reached_t_max(self):
        return self._play_time is None and not self._t_env_reached(self.args.t_max + 1)

    @property
    def _has_not_reached_time_limit(self):
        return self._play_time is not None and (self._end_time - self._start_time) <= self._play_time

    def start(self, play_time_seconds=None, max_iterations=None) -> int:
        if getattr(self.args, "show_exp_parameters", False):
            self.logger.info("Experiment Parameters:\n\n" + pprint.pformat(self.args.__dict__, indent=4, width=1))
        self._play_time = play_time_seconds
        self._init_stepper()
        if self.args.checkpoint_path:
            self.load_models()
            if self.args.evaluate:
                self.evaluate_sequential()
                return 0
        episode = 0
        it = 0
        self._start_time = self._end_time = time.time()
        while self._has_not_reached_time_limit or self._has_not_reached_t_max:
            episode = self._iteration(episode)
            self._end_time = time.time()
            it += 1
            if max_iterations is not None and it >= max_iterations:
                break
        self.stepper.flush()
        self.logger.log_stat("episode", episode, self.stepper.t_env)
        self.stepper.close_env()
        return self.stepper.log_t

    def _iteration(self, episode: int) -> int:
        """One iteration of the training loop (ma_experiment.py:151-175): a train-mode run + at most one train,
        then the test / save / log interval checks. Returns the next episode number."""
        self._train_episode(episode_num=episode)
        if self._t_env_reached(self.last_test_T + self.args.test_interval):
            self._test(max(1, self.args.test_nepisode // self.stepper.batch_size))
        if self.args.save_model and (self.model_save_time == 0
                                     or self._t_env_reached(self.model_save_time + self.args.save_model_interval)):
            self.save_models()
        episode += self.args.batch_size_run
        if self._t_env_reached(self.last_log_T + self.args.log_interval):
            self.logger.log_stat("episode", episode, self.stepper.t_env)
            if hasattr(self.logger, "log_report"):
                self.logger.log_report()
            self.last_log_T = self.stepper.t_env
        return episode

    def _train_episode(self, episode_num):
        episode_batch, env_info = self.stepper.run(test_mode=False)
        if self.on_episode_end is not None:
            self.on_episode_end(env_info)
        self.home_buffer.insert_episode_batch(episode_batch)
        self._train_home(episode_num)

    def _train_home(self, episode_num):
        """Sample + one QLearner.train when the buffer can sample (ma_experiment.py:229-241)."""
        if self.home_buffer.can_sample(self.args.batch_size):
            if str(self.home_buffer.device) == str(self.args.device) and getattr(self.args, "sample_in_place", True):
                # device buffer: the learner reads the sampled episodes in place over their full stored length
                # (steps past max_t_filled are masked out, so loss and gradients equal the truncated batch's),
                # and t_env resolves only after the learner is queued -- no host sync between the launches
                sample = self.home_buffer.sample(self.args.batch_size, view=True)
                self.home_learner.train(sample, LazyTEnv(self.stepper), episode_num)
                return
            sample = self.home_buffer.sample(self.args.batch_size)
            max_ep_t = int(sample.max_t_filled())
            sample = sample[:, :max_ep_t]
            if str(sample.device) != str(self.args.device):
                sample.to(self.args.device)
            self.home_learner.train(sample, self.stepper.t_env, episode_num)

    def _test(self, n_test_runs):
        self.last_test_T = self.stepper.t_env
        for _ in range(n_test_runs):
            self.stepper.run(test_mode=True)

    def evaluate_sequential(self, test_n_episode=None):
        n = self.args.test_nepisode if test_n_episode is None else test_n_episode
        self._init_stepper()
        for _ in range(n):
            self.stepper.run(test_mode=True)

    def save_models(self, identifier=None):
        self.model_save_time = self.stepper.t_env
        path = os.path.join(getattr(self.args, "log_dir", "results"), "models",
                            getattr(self.args, "unique_token", "run"), identifier or "", str(self.model_save_time))
        os.makedirs(path, exist_ok=True)
        for learner in self.learners:
            learner.save_models(path, learner.name)
        return path

    def load_models(self):
        path, step = find_latest_model_path(self.args.checkpoint_path, self.args.load_step)
        for learner in self.learners:
            learner.load_models(path)
        self.stepper.t_env = step
