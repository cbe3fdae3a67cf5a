"""Self-play steppers (API of src/steppers/self_play_parallel_stepper.py:14-201 and
src/steppers/self_play_stepper.py:9-147).

Both plan teams are policy-controlled: the home MAC acts for the first team, a frozen away MAC for the
second (the reference hands the opponent's actions to the env as ``cat(home, away)``,
self_play_parallel_stepper.py:108). One launch of ``mlg_rollout_selfplay`` runs the whole batched
episode with both policies: each side's agents use their own weights and epsilon and are recorded into
their own EpisodeBatch (obs / avail of that side's agents, the shared global state, ``reward[0]`` for
home and ``reward[1]`` for away; stepper_utils.build_pre_transition_data, stepper_utils.py:4-24).
``run()`` returns ``(home_batch, away_batch, env_infos)`` like the reference.
"""
from __future__ import annotations

import torch

from .. import _native
from ..components.batch_view import mlg_batch
from ..components.replay_buffer import RingEpisodeBatch
from ..exceptions import MultiAgentControllerNotInitialized
from .parallel_stepper import LazyEnvInfos, ParallelStepper


class SelfPlayParallelStepper(ParallelStepper):
    # zero-copy run summaries as ParallelStepper: the league's record_runs kernel reads each run's wins straight from
    # the pinned summary slot (LeagueInstance.play -> last_run_info)

    def __init__(self, args, logger, log_start_t=0):
        super().__init__(args, logger, log_start_t)
        if self.spec.n_policy_teams != 2 or self.spec.n_agents % 2:
            raise ValueError(f"A total of {self.spec.n_agents} agents in the env do not fit in the symmetric "
                             "two-team scenario. Ensure the Self-Play scenario has two teams set to is_scripted=False")
        self.away_batch = None
        self._away_buf = None

    def initialize(self, scheme, groups, preprocess, home_mac, away_mac=None):
        if away_mac is None:
            raise ValueError("self-play needs an away MAC (initialize(..., home_mac, away_mac))")
        ParallelStepper.initialize(self, scheme, groups, preprocess, home_mac)
        self.away_mac = away_mac
        self._away_buf = None

    @property
    def epsilons(self):
        return (getattr(self.home_mac.action_selector, "epsilon", None),
                getattr(self.away_mac.action_selector, "epsilon", None))

    def _epsilon_of(self, mac, test_mode):
        return self._epsilon(mac, test_mode)

    def run(self, test_mode=False):
        if self.home_mac is None or self.away_mac is None:
            raise MultiAgentControllerNotInitialized()
        self.reset()
        self.logger.test_mode = test_mode
        self.home_mac.init_hidden(batch_size=self.batch_size)
        self.away_mac.init_hidden(batch_size=self.batch_size)
        eps_h = self._epsilon_of(self.home_mac, test_mode)
        eps_a = self._epsilon_of(self.away_mac, test_mode)
        keep = []
        ring = self._ring if not test_mode else None
        if ring is not None and ring.has_outstanding():
            # the previous train-mode run's episodes still occupy the ring's next slots (not inserted yet):
            # this run goes to a fresh batch, as in the reference, which leaves the buffer untouched until insert
            ring = None
        if ring is not None:
            slot0 = ring.buffer_index
            mb_h, k = mlg_batch(ring)
            keep.append(k)
            mb_h.B, mb_h.ring_slot0, mb_h.ring_size, mb_h.full_write = self.batch_size, slot0, ring.buffer_size, 1
            mb_h.slot_extent = ring.extent_ptr()
            self.home_batch = RingEpisodeBatch(ring, slot0, self.batch_size)
        else:
            self.home_batch = self.new_batch_fn()
            mb_h, k = mlg_batch(self.home_batch)
            keep.append(k)
        if getattr(self.args, "reuse_away_batch", True):
            # one away batch, rewritten in full-write mode by every run (every byte of its B slots is stored,
            # zeros past each episode's end): no per-run allocation and ~1 GB zero fill. The batch returned by
            # run k is therefore overwritten by run k + 1; reuse_away_batch=False gives the reference's fresh
            # batch per run (self_play_parallel_stepper.py:95).
            if self._away_buf is None:
                self._away_buf = self.new_batch_fn()
                # rows of each slot that may be non-zero (T1 = unknown): later runs zero only what the slot's
                # previous episode wrote past the new episode's end
                self._away_extent = torch.full((self.batch_size,), self.episode_limit + 1, dtype=torch.int32,
                                               device=self.device)
            self.away_batch = self._away_buf
            mb_a, k = mlg_batch(self.away_batch)
            mb_a.full_write = 1
            mb_a.slot_extent = self._away_extent.data_ptr()
        else:
            self.away_batch = self.new_batch_fn()
            mb_a, k = mlg_batch(self.away_batch)
        keep.append(k)
        h_agent, a_agent = self.home_mac.agent, self.away_mac.agent
        d, d_a = h_agent.dims(), a_agent.dims()
        if any(getattr(d, f) != getattr(d_a, f) for f, _ in d._fields_):
            raise ValueError("home and away agents must have the same architecture")
        st = self.envs.to_c()
        run_info = self._run_info()
        p_h, p_a = h_agent.packed(), a_agent.packed()  # re-packs (parameters changed) before the timed window
        ev = None
        if self._timed_launch():
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        _native.call("mlg_rollout_selfplay", _native.byref(self._cspec), _native.byref(st), _native.byref(d),
                     _native.ptr(p_h), _native.ptr(p_a), _native.byref(mb_h),
                     _native.byref(mb_a), _native.byref(run_info), float(eps_h), float(eps_a),
                     int(bool(test_mode)), _native.stream_ptr(self.device))
        if ev is not None:
            ev[1].record()
            self.timing.append(ev)
            self._last_end_ev = ev[1]
        del keep
        self._queue_summary(test_mode)
        self._finish_post()
        return self.home_batch, self.away_batch, LazyEnvInfos(self, self._run_id)


class SelfPlayStepper(SelfPlayParallelStepper):
    """Single-env self-play stepper (self_play_stepper.py:9-147): B = 1, returns the final env_info dict."""

    def __init__(self, args, logger, log_start_t=0):
        assert args.batch_size_run == 1
        super().__init__(args, logger, log_start_t)

    def run(self, test_mode=False):
        home, away, infos = super().run(test_mode)
        eh, ea = self.epsilons
        self.logger.log_stat("home_epsilon", eh, self.log_t)
        self.logger.log_stat("away_epsilon", ea, self.log_t)
        return home, away, infos[-1]
