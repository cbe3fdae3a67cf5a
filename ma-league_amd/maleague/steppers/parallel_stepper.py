"""Batched rollout of B envs (API of src/steppers/parallel_stepper.py:14-220).

The reference forks one EnvWorker process per env and exchanges pickled dicts over Queues every step
(env_worker_process.py:27-71); here one launch of the fused gfx950 kernel (mlg_rollout) runs a whole
episode of all B envs: env step, observation, masks, the DRQN agent step and epsilon-greedy
selection, writing the EpisodeBatch tensors in HBM directly. The host reads back one small per-env
summary (episode length, return, won/draw) for t_env and the logger.
"""
from __future__ import annotations

from collections import deque
from collections.abc import Sequence
from functools import partial

import numpy as np
import torch

from .. import _native
from ..components.batch_view import mlg_batch
from ..components.episode_batch import EpisodeBatch
from ..components.replay_buffer import RingEpisodeBatch
from ..custom_logging import Collectibles, Originator
from ..envs.teams_env import TeamsEnvSpec, VecEnvState
from ..exceptions import MultiAgentControllerNotInitialized


def _same_device(a, b) -> bool:
    a, b = torch.device(a), torch.device(b)
    if a.type != b.type:
        return False
    if a.type == "cuda":
        cur = torch.cuda.current_device()
        return (cur if a.index is None else a.index) == (cur if b.index is None else b.index)
    return True


class EnvInfos(Sequence):
    """The per-run list of env_info dicts (``{"battle_won": [home, away], "draw": bool}``) in order of
    termination (parallel_stepper.py:124,183-184: by episode length, then env index), materialised on access: a plain
    list of 4096 dicts per run costs milliseconds of host time, and the ordering itself is computed on first access."""

    def __init__(self, won, draw, ep_len):
        self._won, self._draw, self._len, self._order = won, draw, ep_len, None

    def _o(self):
        if self._order is None:
            self._order = np.lexsort((np.arange(len(self._len)), self._len))
        return self._order

    @property
    def won(self):
        return self._won[self._o()]

    @property
    def draw(self):
        return self._draw[self._o()]

    def __len__(self):
        return len(self._draw)

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[k] for k in range(*i.indices(len(self)))]
        k = self._o()[i]
        return {"battle_won": [bool(self._won[k, 0]), bool(self._won[k, 1])], "draw": bool(self._draw[k])}


class LazyEnvInfos(Sequence):
    """env_infos of a run whose summary is still in flight: resolves (waits for the rollout) on first use."""

    def __init__(self, stepper, run_id):
        self._stepper, self._run_id, self._infos = stepper, run_id, None

    def _get(self):
        if self._infos is None:
            self._infos = self._stepper._env_infos_of(self._run_id)
        return self._infos

    def __len__(self):
        return self._stepper.batch_size

    def __getitem__(self, i):
        return self._get()[i]


class EnvStepper:
    def __init__(self, args, logger, log_start_t=0):
        self.args = args
        self.logger = logger
        self.batch_size = None
        self.t_env = 0
        self.is_initalized = False  # [sic] reference attribute name (ma_experiment.py:124)
        self.log_start_t = log_start_t or 0

    @property
    def log_t(self):
        return self.log_start_t + self.t_env


class ParallelStepper(EnvStepper):
    def __init__(self, args, logger, log_start_t=0):
        super().__init__(args, logger, log_start_t)
        self.batch_size = args.batch_size_run
        self.device = torch.device(args.device)
        env_args = dict(args.env_args)
        env_args.setdefault("seed", getattr(args, "seed", 0))
        self.spec = self._build_spec(env_args, getattr(args, "config_dir", None))
        self.policy_team_id = self.spec.policy_team
        self.env_info = self.spec.env_info()
        self.episode_limit = self.env_info["episode_limit"]
        self._cspec = self.spec.to_c()
        self.envs = VecEnvState(self.spec, self.batch_size, self.device)
        B = self.batch_size
        # one int32 buffer for the per-run summary -> one D2H copy per run:
        # [ep_len B | won 2B | draw B | return B (f32 bits) | away return B (f32 bits, self-play)]
        self._info = torch.zeros(6 * B, dtype=torch.int32, device=self.device)
        # running count of agent rows the rollout kernels pushed through the MFMA cell (diagnostics / bench)
        self.agent_rows = torch.zeros(1, dtype=torch.int64, device=self.device)
        pin = self.device.type == "cuda"
        # run summaries in flight: one pinned host buffer per run, up to _HOST_RING runs unresolved
        self._info_hosts = [torch.zeros(6 * B, dtype=torch.int32, pin_memory=pin) for _ in range(self._HOST_RING)]
        self._pendings = deque()  # (run_id, event, test_mode, host buffer): summary copies in flight
        self._last_end_ev = None  # end event of the last timed launch (bench.py): reused as its summary event
        self._host_slot = None  # zero-copy: the pinned ring slot of the last launched run
        self._post = []       # resolved runs awaiting host post-processing (logger, env_infos)
        self._runs = {}       # run_id -> (last_run dict, EnvInfos), the latest two
        self._run_id = 0
        self._t = 0
        self.env_steps_this_run = 0
        self.new_batch_fn = None
        self.home_mac = None
        self.home_batch = None
        self.away_mac = None  # self-play only (SelfPlayParallelStepper)
        self.timing = None  # list -> (start, end) HIP events around rollout launches (bench.py)
        self.timing_every = 1  # time every k-th launch only (an event pair costs a few us of GPU queue time)
        self.t_history = None  # list -> (run_id, longest episode) of every resolved run (bench.py latency floor)
        self._launches = 0
        self._ring = None   # ReplayBuffer written in place (zero-copy insert), see attach_replay()

    _batch_keys = ("state", "obs", "actions", "avail_actions", "reward", "terminated", "actions_onehot", "filled")
    _HOST_RING = 4
    # zero-copy summaries: the rollout kernel writes the run summary straight into the pinned host buffer of the
    # ring (device-accessible on ROCm) instead of a device buffer plus an async D2H blit -- the blit and its
    # cross-queue signals cost ~20 us of GPU idle per run. The self-play steppers keep the device buffer: the league
    # reads the run's wins on the device (LeagueInstance.play -> DistributedLeague.record_runs).
    _ZERO_COPY = True

    def _build_spec(self, env_args, config_dir):
        return TeamsEnvSpec.from_env_args(env_args, config_dir)

    def set_match_build_plan(self, plan):
        """Swap the env's team rosters between runs (a league match: home team vs the adversary's team,
        league_experiment_process.py:57-62, where the reference rebuilds the whole experiment and its env). The new
        plan must keep the env's shape (units, agents, actions, policy team) -- the batches, replay buffer and MACs
        stay valid; the roles / attack types of every unit follow the plan. The spec travels by value as a kernel
        argument, so runs already queued keep the rosters they were launched with."""
        env_args = dict(self.args.env_args)
        env_args["match_build_plan"] = plan
        env_args.setdefault("seed", getattr(self.args, "seed", 0))
        spec = self._build_spec(env_args, getattr(self.args, "config_dir", None))
        old = self.spec
        if (spec.U, spec.n_agents, spec.n_actions, spec.policy_team, spec.n_policy_teams) != \
                (old.U, old.n_agents, old.n_actions, old.policy_team, old.n_policy_teams):
            raise ValueError(f"match_build_plan changes the env shape (U {old.U} -> {spec.U}, agents {old.n_agents} -> "
                             f"{spec.n_agents}, policy teams {old.n_policy_teams} -> {spec.n_policy_teams}): a "
                             "roster swap keeps the team sizes")
        self.args.env_args = env_args
        self.spec = spec
        self.envs.spec = spec
        self._cspec = spec.to_c()

    def _to_mlg(self, batch):
        return mlg_batch(batch)

    def _rollout(self, mb, run_info, epsilon, test_mode):
        agent = self.home_mac.agent
        st = self.envs.to_c()
        _native.call("mlg_rollout", _native.byref(self._cspec), _native.byref(st), _native.byref(agent.dims()),
                     _native.ptr(agent.packed()), _native.byref(mb), _native.byref(run_info), float(epsilon),
                     int(bool(test_mode)), _native.stream_ptr(self.device))

    def initialize(self, scheme, groups, preprocess, home_mac, away_mac=None):
        if away_mac is not None:
            raise NotImplementedError("ParallelStepper drives one policy; self-play (home + away MAC) is "
                                      "SelfPlayParallelStepper (steppers.SELF_REGISTRY['parallel'])")
        self.new_batch_fn = partial(EpisodeBatch, scheme, groups, self.batch_size, self.episode_limit + 1,
                                    preprocess=preprocess, device=self.device)
        self.home_mac = home_mac
        self.is_initalized = True

    def get_env_info(self):
        return self.env_info

    # ---- the run summary travels back asynchronously; host state resolves on first use --------------
    # Nothing in a training iteration needs the host to wait for the GPU: the epsilon of the next run is exact
    # without the previous run's episode lengths once the schedule is flat over every t_env still possible
    # (t_env_bounds), the learner's log check likewise, so the host runs up to _HOST_RING runs ahead and a
    # slow or contended host core does not stall the device (one process per GPU, eight per node).
    @property
    def t_env(self) -> int:
        self._resolve()
        return self._t_env

    @t_env.setter
    def t_env(self, value: int):
        if getattr(self, "_pendings", None):
            self._resolve()
        self._t_env = int(value)

    @property
    def t(self) -> int:
        self._resolve()
        return self._t

    @t.setter
    def t(self, value: int):
        self._t = int(value)

    @property
    def last_run(self):
        self._resolve()
        self._finish_post()
        return self._runs[self._run_id][0] if self._run_id in self._runs else None

    def t_env_bounds(self):
        """(lower, upper) bounds of t_env without waiting: the resolved value, plus B * episode_limit per
        train-mode run still in flight."""
        lo = self._t_env
        pend = sum(1 for p in self._pendings if not p[2])
        return lo, lo + pend * self.batch_size * self.episode_limit

    def _epsilon(self, mac, test_mode):
        """action_selector.epsilon = schedule.eval(t_env) (parallel_stepper.py / basic_controller semantics),
        resolved on the host only while the (monotone) schedule still changes inside t_env_bounds()."""
        sel = mac.action_selector
        lo, hi = self.t_env_bounds()
        e = sel.schedule.eval(lo)
        if hi != lo and sel.schedule.eval(hi) != e:
            e = sel.schedule.eval(self.t_env)
        sel.epsilon = e
        if test_mode:
            sel.epsilon = 0.0
            return 0.0
        return float(e)

    def _zero_copy(self) -> bool:
        return self._ZERO_COPY and self.device.type == "cuda"

    def _reserve_host(self):
        """The ring's pinned buffer for the next run (the oldest run in flight is resolved first when all are
        taken)."""
        while len(self._pendings) >= self._HOST_RING:
            self._resolve_one()
        return self._info_hosts[(self._run_id + 1) % self._HOST_RING]

    def _queue_summary(self, test_mode):
        """Zero-copy: the kernel already wrote the summary into the reserved pinned buffer; an event marks its
        completion. Else async D2H of the device summary into a pinned buffer of the ring (stream-ordered before
        the next run's kernel rewrites the device copy), then the event."""
        ev = None
        if self._zero_copy():
            host = self._host_slot
            # the run's timing end event (bench.py) already marks the kernel's completion: no second event record
            # (each costs a few us of queue time between the rollout and the learner)
            ev = self._last_end_ev
        else:
            host = self._reserve_host()
            host.copy_(self._info, non_blocking=True)
        self._last_end_ev = None
        if ev is None:
            ev = torch.cuda.Event()
            ev.record()
        self._run_id += 1
        self._pendings.append((self._run_id, ev, test_mode, host))

    def _resolve(self):
        """Wait for every run in flight (t_env, t); the rest of the host work is deferred."""
        while getattr(self, "_pendings", None):
            self._resolve_one()

    def _resolve_one(self):
        run_id, ev, test_mode, buf = self._pendings.popleft()
        ev.synchronize()
        B = self.batch_size
        host = buf.numpy().copy()
        ep_len = host[0:B]
        self._t = int(ep_len.max())
        if self.t_history is not None:
            self.t_history.append((run_id, self._t))
        if not test_mode:
            self.env_steps_this_run = int(ep_len.sum())
            self._t_env += self.env_steps_this_run
        self._post.append((run_id, host, self._t, self._t_env, test_mode))

    def _finish_post(self):
        B = self.batch_size
        mode_now = self.logger.test_mode
        for run_id, host, t_max, t_env, test_mode in self._post:
            self.logger.test_mode = test_mode  # the run's mode (its summary may resolve after a later run())
            ep_len = host[0:B]  # host is this run's own copy of the summary ring slot (_resolve_one)
            won = host[B:3 * B].reshape(B, 2) != 0
            draw = host[3 * B:4 * B] != 0
            ret = host[4 * B:5 * B].view(np.float32)
            ret_away = host[5 * B:6 * B].view(np.float32)
            # env_infos in order of termination (EnvInfos: ordered on first access)
            infos = EnvInfos(won, draw, ep_len)
            last = {"ep_len": torch.from_numpy(ep_len), "returns": torch.from_numpy(ret)}
            if self.away_mac is not None:
                last["away_returns"] = torch.from_numpy(ret_away)
            self._runs[run_id] = (last, infos)
            self._runs.pop(run_id - 2, None)
            # the per-run arrays go to the logger as arrays (listed at log time); float32 returns list as the same
            # Python floats as their float64 copies. The won / draw ratios are order-free integer sums, so they are
            # collected in env order rather than termination order.
            self.logger.collect(Collectibles.RETURN, ret, origin=Originator.HOME, parallel=True)
            if self.away_mac is not None:
                self.logger.collect(Collectibles.RETURN, ret_away, origin=Originator.AWAY, parallel=True)
            self.logger.collect(Collectibles.WON, won[:, 0], origin=Originator.HOME, parallel=True)
            self.logger.collect(Collectibles.WON, won[:, 1], origin=Originator.AWAY, parallel=True)
            self.logger.collect(Collectibles.DRAW, draw, parallel=True)
            self.logger.collect(Collectibles.STEPS, t_max, parallel=True)
            self.logger.log(t_env)
        self.logger.test_mode = mode_now
        self._post = []

    def _env_infos_of(self, run_id):
        self._resolve()
        self._finish_post()
        if run_id not in self._runs:
            raise RuntimeError("env_infos of an old run are no longer available")
        return self._runs[run_id][1]

    def flush(self):
        """Resolve and post-process every run launched so far."""
        self._resolve()
        self._finish_post()

    def attach_replay(self, buffer) -> bool:
        """Let train-mode runs write their episodes straight into `buffer`'s next slots (the buffer's
        insert_episode_batch then only advances its indices). Returns False when the layouts differ."""
        ok = (_same_device(buffer.device, self.device) and buffer.max_seq_length == self.episode_limit + 1
              and buffer.buffer_size >= self.batch_size
              and all(k in buffer.data.transition_data for k in self._batch_keys))
        self._ring = buffer if ok else None
        return ok

    def save_replay(self):
        pass

    def close_env(self):
        pass

    def reset(self):
        pass  # per-run host state resolves lazily (_resolve_one); nothing to wait for before a launch

    def _launch(self, batch: EpisodeBatch, epsilon: float, test_mode: bool):
        mb, keep = self._to_mlg(batch)
        self._launch_mb(mb, epsilon, test_mode)
        del keep

    def last_run_info(self) -> torch.Tensor:
        """The int32 [6 B] summary the last launched run writes (ep_len | won [B, 2] | draw | ret | ...): its pinned
        ring slot in zero-copy mode (device-accessible, read by stream-ordered kernels such as the league's
        record_runs), else the device buffer."""
        return self._host_slot if self._zero_copy() and self._host_slot is not None else self._info

    def _run_info(self):
        B = self.batch_size
        if self._zero_copy():
            self._host_slot = self._reserve_host()
            info = self._host_slot
        else:
            info = self._info
        return _native.MlgRunInfo(info[0:B].data_ptr(), info[4 * B:5 * B].data_ptr(), info[B:3 * B].data_ptr(),
                                  info[3 * B:4 * B].data_ptr(), self.agent_rows.data_ptr(),
                                  info[5 * B:6 * B].data_ptr())

    def _timed_launch(self) -> bool:
        self._launches += 1
        return self.timing is not None and self.timing_every > 0 and self._launches % self.timing_every == 0

    def _launch_mb(self, mb, epsilon: float, test_mode: bool):
        run_info = self._run_info()
        self.home_mac.agent.packed()  # a re-pack (parameters changed) runs before the timed window
        ev = None
        if self._timed_launch():
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        self._rollout(mb, run_info, epsilon, test_mode)
        if ev is not None:
            ev[1].record()
            self.timing.append(ev)
            self._last_end_ev = ev[1]

    def run(self, test_mode=False):
        if self.home_mac is None:
            raise MultiAgentControllerNotInitialized()
        self.reset()
        self.logger.test_mode = test_mode
        self.home_mac.init_hidden(batch_size=self.batch_size)
        eps = self._epsilon(self.home_mac, test_mode)
        ring = self._ring if not test_mode else None
        if ring is not None and ring.has_outstanding():
            # the previous train-mode run's episodes still occupy the ring's next slots (not inserted yet):
            # this run goes to a fresh batch, as in the reference, which leaves the buffer untouched until insert
            ring = None
        if ring is not None:
            slot0 = ring.buffer_index
            mb, keep = self._to_mlg(ring)
            # full-write mode: the kernel writes every byte of the B ring slots (zeros past each episode's end,
            # by the idle lanes of finished envs), so nothing is zero-initialised or copied
            mb.B, mb.ring_slot0, mb.ring_size, mb.full_write = self.batch_size, slot0, ring.buffer_size, 1
            mb.slot_extent = ring.extent_ptr()
            self._launch_mb(mb, eps, test_mode)
            del keep
            self.home_batch = RingEpisodeBatch(ring, slot0, self.batch_size)
        else:
            self.home_batch = self.new_batch_fn()
            self._launch(self.home_batch, eps, test_mode)
        # summary of this run: async D2H into pinned memory; t_env / env_infos resolve on first use, the
        # earlier runs' host post-processing runs now, while this rollout is on the GPU
        self._queue_summary(test_mode)
        self._finish_post()
        return self.home_batch, LazyEnvInfos(self, self._run_id)


class EpisodeStepper(ParallelStepper):
    """Single-env stepper (src/steppers/episode_stepper.py:16-186): same kernel with B = 1; returns the
    final env_info dict instead of a list."""

    def __init__(self, args, logger, log_start_t=0):
        assert args.batch_size_run == 1
        super().__init__(args, logger, log_start_t)

    @property
    def epsilon(self):
        return getattr(self.home_mac.action_selector, "epsilon", None)

    def run(self, test_mode=False):
        batch, infos = super().run(test_mode)
        self.logger.log_stat("home_epsilon", self.epsilon, self.log_t)
        return batch, infos[-1]
