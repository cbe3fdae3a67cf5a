"""Generate golden vectors from the reference (PMatthaei/ma-league) for the hot path.

TEST INFRASTRUCTURE ONLY. Runs in the build container, where the reference is mounted read-only
at /root/reference. It imports the reference's own Python modules (PYTHONPATH=/root/reference/src)
and records their inputs/outputs as small .npz fixtures (data only, no reference source text).
The GPU box never sees the reference: it reads the committed .npz files.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Fixtures (all float32/int64 arrays; dict keys documented per function below):
  drqn_step.npz        DRQNAgentNetwork.forward            src/marl/modules/agents/drqn_agent.py:29-35
  mac_forward.npz      BasicMAC._build_inputs + forward    src/marl/controllers/basic_controller.py:38-50,80-92
  eps_greedy.npz       EpsilonGreedyActionSelector.select  src/marl/components/action_selectors.py:44-62 (test_mode)
                       DecayThenFlatSchedule.eval          src/marl/components/epsilon_schedules.py:21-25
  qmix_fwd.npz         QMixer.forward                      src/marl/modules/mixers/qmix.py:41-59
  qlearner_*.npz       QLearner.train (3 consecutive calls) src/marl/learners/q_learner.py:34-131
  replay_buffer.npz    ReplayBuffer insert/sample/max_t    src/marl/components/replay_buffers/replay_buffer.py:22-53
  parallel_stepper.npz ParallelStepper.run bookkeeping     src/steppers/parallel_stepper.py:82-216
                       (fake env with scripted termination; probe shims listed in _stepper_fixture)
  pfsp.npz             PayoffWrapper.win_rates + PFSPSampling weightings
                       src/league/components/payoff_entry.py:23-30, src/league/components/self_play.py:49-65
  checkpoint.npz       QLearner.save_models/load_models resume  src/marl/learners/q_learner.py:133-147
  logger.npz           MainLogger collect/log aggregation  src/custom_logging/logger.py:24-173
  ckpt_qmix/100/*.th   the reference's own checkpoint files (torch.save of state dicts; tests load them
                       with weights_only=True)
"""
import collections
import collections.abc
import functools
import importlib.util
import os
import sys
import types
from types import SimpleNamespace

import numpy as np

REF_SRC = "/root/reference/src"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REF_SRC)
sys.dont_write_bytecode = True

import torch as th  # noqa: E402

th.set_num_threads(1)

from marl.components.episode_batch import EpisodeBatch  # noqa: E402
from marl.components.transforms import OneHot  # noqa: E402
from marl.components.action_selectors import EpsilonGreedyActionSelector  # noqa: E402
from marl.components.epsilon_schedules import DecayThenFlatSchedule  # noqa: E402
from marl.components.replay_buffers.replay_buffer import ReplayBuffer  # noqa: E402
from marl.controllers.basic_controller import BasicMAC  # noqa: E402
from marl.modules.agents.drqn_agent import DRQNAgentNetwork  # noqa: E402
from marl.modules.mixers.qmix import QMixer  # noqa: E402
from marl.learners.q_learner import QLearner  # noqa: E402


def base_args(**kw):
    a = dict(n_agents=5, n_actions=15, state_shape=60, rnn_hidden_dim=64, obs_last_action=True,
             obs_agent_id=True, agent="rnn", agent_output_type="q", action_selector="epsilon_greedy",
             epsilon_start=1.0, epsilon_finish=0.05, epsilon_anneal_time=50000, freeze_native=False,
             device="cpu", mixer="qmix", mixing_embed_dim=32, hypernet_layers=2, hypernet_embed=64,
             double_q=True, gamma=0.99, lr=0.0005, optim_alpha=0.99, optim_eps=1e-5, grad_norm_clip=10,
             target_update_interval=200, learner_log_interval=0)
    a.update(kw)
    return SimpleNamespace(**a)


def sd_to_np(prefix, sd):
    return {f"{prefix}{k}": v.detach().cpu().numpy().copy() for k, v in sd.items()}


def scheme_for(d_obs, n_actions, state_shape):
    # Same scheme as MultiAgentExperiment._build_schemes (src/runs/train/ma_experiment.py:99-118)
    scheme = {
        "state": {"vshape": state_shape},
        "obs": {"vshape": d_obs, "group": "agents"},
        "actions": {"vshape": (1,), "group": "agents", "dtype": th.long},
        "avail_actions": {"vshape": (n_actions,), "group": "agents", "dtype": th.int},
        "reward": {"vshape": (1,)},
        "terminated": {"vshape": (1,), "dtype": th.uint8},
    }
    groups = {"agents": 5}
    preprocess = {"actions": ("actions_onehot", [OneHot(out_dim=n_actions)])}
    return scheme, groups, preprocess


# ----------------------------------------------------------------------------------------------
def drqn_fixture():
    th.manual_seed(0)
    args = base_args()
    agent = DRQNAgentNetwork(100, args)
    g = th.Generator().manual_seed(1)
    inputs = th.randn(40, 100, generator=g)
    hidden = th.randn(40, 64, generator=g) * 0.5
    with th.no_grad():
        q, h = agent(inputs, hidden)
    out = sd_to_np("p.", agent.state_dict())
    out.update(inputs=inputs.numpy(), hidden=hidden.numpy(), q=q.numpy(), h=h.numpy())
    np.savez_compressed(os.path.join(OUT, "drqn_step.npz"), **out)


def make_batch(B, T, N, d_obs, A, S, lengths, seed, device="cpu"):
    """A scheme-conforming EpisodeBatch with episodes of the given lengths (steps)."""
    scheme, groups, preprocess = scheme_for(d_obs, A, S)
    groups = {"agents": N}
    batch = EpisodeBatch(scheme, groups, B, T, preprocess=preprocess, device=device)
    rng = np.random.RandomState(seed)
    for b, L in enumerate(lengths):
        for t in range(min(L + 1, T)):
            avail = (rng.rand(N, A) < 0.6).astype(np.int32)
            for n in range(N):
                if avail[n].sum() == 0:
                    avail[n, rng.randint(A)] = 1
            acts = np.array([[rng.choice(np.nonzero(avail[n])[0])] for n in range(N)], dtype=np.int64)
            pre = {"state": [rng.randn(S).astype(np.float32).tolist()],
                   "avail_actions": [avail.tolist()],
                   "obs": [rng.randn(N, d_obs).astype(np.float32).tolist()]}
            batch.update(pre, bs=[b], ts=t, mark_filled=True)
            batch.update({"actions": th.tensor(acts).unsqueeze(0)}, bs=[b], ts=t, mark_filled=False)
            if t < L:
                post = {"reward": [(float(rng.randn()),)], "terminated": [(t == L - 1,)]}
                batch.update(post, bs=[b], ts=t, mark_filled=False)
    return batch, scheme, groups, preprocess


def batch_to_np(prefix, batch):
    return {f"{prefix}{k}": v.cpu().numpy().copy() for k, v in batch.data.transition_data.items()}


def mac_fixture():
    th.manual_seed(2)
    args = base_args()
    B, T, N, d_obs, A, S = 3, 4, 5, 80, 15, 60
    batch, scheme, groups, preprocess = make_batch(B, T, N, d_obs, A, S, [3, 2, 3], seed=3)
    mac = BasicMAC(batch.scheme, groups, args)
    mac.init_hidden(B)
    qs = []
    with th.no_grad():
        for t in range(T):
            qs.append(mac.forward(batch, t).numpy().copy())
    out = sd_to_np("p.", mac.agent.state_dict())
    out.update(batch_to_np("b.", batch))
    out["q"] = np.stack(qs)
    np.savez_compressed(os.path.join(OUT, "mac_forward.npz"), **out)


def eps_fixture():
    args = base_args()
    sel = EpsilonGreedyActionSelector(args)
    rng = np.random.RandomState(4)
    B, N, A = 6, 5, 15
    q = rng.randn(B, N, A).astype(np.float32)
    avail = (rng.rand(B, N, A) < 0.5).astype(np.int32)
    avail[..., 0] = np.maximum(avail[..., 0], (avail.sum(-1) == 0))
    # crafted cases: exact ties (first index must win), unavailable max, single available action
    q[0, 0, :] = 1.0
    avail[0, 0, :] = 1
    q[0, 1, 3] = q[0, 1, 7] = 5.0
    avail[0, 1, :] = 1
    q[1, 0, :] = np.arange(A, dtype=np.float32)
    avail[1, 0, :] = 0
    avail[1, 0, 2] = 1
    q[1, 1, 14] = 100.0
    avail[1, 1, 14] = 0
    avail[1, 1, 13] = 1
    q[2, 2, :] = -1e30
    avail[2, 2, :] = 1
    acts, greedy = sel.select(th.tensor(q), th.tensor(avail), t_env=0, test_mode=True)
    sched = DecayThenFlatSchedule(1.0, 0.05, 50000, decay="linear")
    ts = np.array([0, 1, 100, 25000, 49999, 50000, 50001, 10 ** 7], dtype=np.int64)
    eps = np.array([sched.eval(int(t)) for t in ts], dtype=np.float64)
    np.savez_compressed(os.path.join(OUT, "eps_greedy.npz"), q=q, avail=avail, actions=acts.numpy(),
                        is_greedy=greedy.numpy(), sched_t=ts, sched_eps=eps)


def qmix_fixture():
    th.manual_seed(5)
    args = base_args()
    mixer = QMixer(args)
    g = th.Generator().manual_seed(6)
    qs = th.randn(4, 6, 5, generator=g)
    st = th.randn(4, 6, 60, generator=g)
    with th.no_grad():
        y = mixer(qs, st)
    out = sd_to_np("p.", mixer.state_dict())
    out.update(agent_qs=qs.numpy(), states=st.numpy(), q_tot=y.numpy())
    np.savez_compressed(os.path.join(OUT, "qmix_fwd.npz"), **out)


class StatLogger:
    def __init__(self):
        self.stats = []

    def log_stat(self, key, value, t):
        self.stats.append((key, float(np.asarray(value)), t))

    def info(self, *a, **k):
        pass


def qlearner_fixture(tag, full, **kw):
    th.manual_seed(7)
    args = base_args(**kw)
    B, T, N, d_obs, A, S = 4, 7, 5, 80, 15, 60
    lengths = [6, 3, 4, 2]
    batch, scheme, groups, preprocess = make_batch(B, T, N, d_obs, A, S, lengths, seed=8)
    mac = BasicMAC(batch.scheme, groups, args)
    logger = StatLogger()
    learner = QLearner(mac, batch.scheme, logger, args, name="home")
    learner.build_optimizer()
    out = {}
    out.update(sd_to_np("p0.agent.", mac.agent.state_dict()))
    if learner.mixer is not None:
        out.update(sd_to_np("p0.mixer.", learner.mixer.state_dict()))
    out.update(batch_to_np("b.", batch))
    calls = [(100, 0), (200, 32), (300, 232)]  # (t_env, episode_num): 3rd call crosses target_update_interval
    out["calls"] = np.array(calls, dtype=np.int64)
    for i, (t_env, ep) in enumerate(calls):
        logger.stats.clear()
        learner.train(batch, t_env, ep)
        stats = {k.replace("home_qlearner_", ""): v for k, v, _ in logger.stats}
        for k in ["loss", "grad_norm", "td_error_abs", "q_taken_mean", "target_mean"]:
            out[f"stat{i}.{k}"] = np.array(stats[k], dtype=np.float64)
        if full or i == len(calls) - 1:
            out.update(sd_to_np(f"p{i + 1}.agent.", mac.agent.state_dict()))
            out.update(sd_to_np(f"p{i + 1}.target_agent.", learner.target_mac.agent.state_dict()))
            if learner.mixer is not None and not isinstance(learner.mixer, type(None)):
                msd = learner.mixer.state_dict()
                if len(msd):
                    out.update(sd_to_np(f"p{i + 1}.mixer.", msd))
    out["trained_steps"] = np.array(mac.agent.trained_steps, dtype=np.int64)
    np.savez_compressed(os.path.join(OUT, f"qlearner_{tag}.npz"), **out)


def replay_fixture():
    B, T, N, d_obs, A, S = 3, 5, 5, 8, 4, 6
    scheme, groups, preprocess = scheme_for(d_obs, A, S)
    groups = {"agents": N}
    buf = ReplayBuffer(scheme, groups, 7, T, preprocess=preprocess, device="cpu")
    out = {}
    for k in range(4):
        batch, *_ = make_batch(B, T, N, d_obs, A, S, [4 - k % 2, 2 + k % 3, 1 + k], seed=10 + k)
        buf.insert_episode_batch(batch)
        out[f"ins{k}.obs"] = batch["obs"].numpy().copy()
        out[f"ins{k}.filled"] = batch["filled"].numpy().copy()
        out[f"after{k}.buffer_index"] = np.array(buf.buffer_index)
        out[f"after{k}.episodes_in_buffer"] = np.array(buf.episodes_in_buffer)
        out[f"after{k}.obs"] = buf["obs"].numpy().copy()
        out[f"after{k}.filled"] = buf["filled"].numpy().copy()
        out[f"after{k}.actions_onehot"] = buf["actions_onehot"].numpy().copy()
    out["max_t_filled"] = np.array(int(buf.max_t_filled()))
    # exactly-full path of sample() returns the first batch_size episodes (replay_buffer.py:48-49)
    buf2 = ReplayBuffer(scheme, groups, 3, T, preprocess=preprocess, device="cpu")
    batch, *_ = make_batch(B, T, N, d_obs, A, S, [2, 3, 1], seed=20)
    buf2.insert_episode_batch(batch)
    smp = buf2.sample(3)
    out["full_sample.obs"] = smp["obs"].numpy().copy()
    out["full_sample.max_t"] = np.array(int(smp.max_t_filled()))
    np.savez_compressed(os.path.join(OUT, "replay_buffer.npz"), **out)


# ----------------------------------------------------------------------------------------------
def _stepper_fixture():
    """Runs the reference ParallelStepper.run loop against a fake env with scripted termination.

    Probe shims (this generator only; none of them is product code):
      * collections.Sized/Mapping aliased (Python 3.10 removed them; custom_logging/logger.py:3)
      * torch.multiprocessing.queue.Queue given its mandatory ctx (parallel_stepper.py:32),
        with put() cloning tensors (removes the reference's shared-memory race on sent actions; see SyncQueue)
      * a fake `envs` module whose REGISTRY builds FakeEnv (maenv is not in the container)
      * custom_logging.platforms stubbed (sacred/tensorboard absent); the stepper only needs the
        Collectibles/Originator enums and a logger object with collect()/log()
    """
    collections.Sized = collections.abc.Sized
    collections.Mapping = collections.abc.Mapping
    import multiprocessing as mp
    import torch.multiprocessing.queue as tq
    ctx = mp.get_context("fork")
    base_queue = tq.Queue

    class SyncQueue(base_queue):
        """Clones tensors at put(): the reference sends views of one float tensor (parallel_stepper.py:126,
        148-149) through torch Queues whose feeder thread moves the storage to shared memory asynchronously,
        which races with the parent's next row write (observed: an env stepping with all-zero actions).
        The intended semantics -- each env receives its own actions -- is what the fixture records."""

        def __init__(self, *a, **k):
            super().__init__(*a, ctx=ctx, **k)

        def put(self, obj, *a, **k):
            if isinstance(obj, tuple):
                obj = tuple(o.clone() if isinstance(o, th.Tensor) else o for o in obj)
            return super().put(obj, *a, **k)

    tq.Queue = SyncQueue

    N, A, d_obs, S, B = 3, 6, 4, 5, 5
    term_at = [3, 1, 5, 2, 5]  # env i terminates when stepping at t == term_at[i]

    class FakeEnv:
        count = 0

        def __init__(self, **kw):
            self.idx = FakeEnv.count
            FakeEnv.count += 1
            self.t = 0

        def _obs(self):
            return [[float(self.idx * 100 + self.t * 10 + n + 0.25 * k) for k in range(d_obs)] for n in range(N)]

        def get_obs(self):
            return self._obs()

        def get_state(self):
            return [float(self.idx * 1000 + self.t * 10 + k) for k in range(S)]

        def get_avail_actions(self):
            return [[1 if (a + n + self.t + self.idx) % 3 != 0 or a == 0 else 0 for a in range(A)]
                    for n in range(N)]

        def step(self, actions):
            self.last_actions = [int(a) for a in actions]
            r = float(self.idx) + 0.5 * self.t + 0.01 * sum(self.last_actions)
            done = self.t == term_at[self.idx]
            self.t += 1
            won = [self.idx % 2 == 0, False]
            return self._obs(), [r, -r], [done, done], {"battle_won": won, "draw": self.idx == 3}

        def reset(self):
            self.t = 0

        def get_env_info(self):
            return {"n_agents": N, "n_actions": A, "state_shape": S, "obs_shape": d_obs, "episode_limit": 8}

        def close(self):
            pass

    envs_mod = types.ModuleType("envs")
    envs_mod.REGISTRY = {"fake": lambda **kw: FakeEnv(**kw)}
    sys.modules["envs"] = envs_mod
    plat = types.ModuleType("custom_logging.platforms")
    plat.CustomSacredLogger = object
    plat.CustomTensorboardLogger = object
    sys.modules["custom_logging.platforms"] = plat
    cons = types.ModuleType("custom_logging.platforms.console")
    cons.CustomConsoleLogger = object
    sys.modules["custom_logging.platforms.console"] = cons
    for name in ["bin", "bin.controls", "bin.controls.headless_controls"]:  # maenv GUI controls (episode_stepper.py:2)
        sys.modules[name] = types.ModuleType(name)
    sys.modules["bin.controls.headless_controls"].HeadlessControls = object

    from steppers.parallel_stepper import ParallelStepper

    class Log:
        def __init__(self):
            self.collected = []
            self.test_mode = False

        def collect(self, key, data, origin=None, parallel=False):
            self.collected.append((key.name, origin.value if origin is not None else None, data))

        def log(self, t):
            self.logged_t = t

    class StubMAC:
        """Deterministic actions: (t*7 + env*3 + agent) % A restricted to available ones."""

        def __init__(self):
            self.calls = []

        def init_hidden(self, batch_size):
            pass

        def select_actions(self, batch, t_ep, t_env, bs=slice(None), test_mode=False):
            avail = batch["avail_actions"][:, t_ep]
            idx = list(range(batch.batch_size))[bs] if isinstance(bs, slice) else list(bs)
            self.calls.append((t_ep, list(idx)))
            acts = []
            for e in idx:
                row = []
                for n in range(N):
                    a = (t_ep * 7 + e * 3 + n) % A
                    while avail[e, n, a] == 0:
                        a = (a + 1) % A
                    row.append(a)
                acts.append(row)
            return th.tensor(acts, dtype=th.long), None

    args = SimpleNamespace(batch_size_run=B, env="fake", device="cpu",
                           env_args={"match_build_plan": [{"is_scripted": True}, {"is_scripted": False}]})
    log = Log()
    stepper = ParallelStepper(args, log)
    scheme, groups, preprocess = scheme_for(d_obs, A, S)
    groups = {"agents": N}
    mac = StubMAC()
    stepper.initialize(scheme, groups, preprocess, mac)
    out = {"term_at": np.array(term_at)}
    for run in range(2):
        test_mode = run == 1
        batch, infos = stepper.run(test_mode=test_mode)
        for k, v in batch.data.transition_data.items():
            out[f"run{run}.{k}"] = v.numpy().copy()
        out[f"run{run}.t_env"] = np.array(stepper.t_env)
        out[f"run{run}.t"] = np.array(stepper.t)
        out[f"run{run}.info_won0"] = np.array([i["battle_won"][0] for i in infos])
        out[f"run{run}.info_draw"] = np.array([i["draw"] for i in infos])
        ret = [c for c in log.collected if c[0] == "RETURN"][-1][2]
        out[f"run{run}.returns"] = np.array(ret, dtype=np.float64)
        steps = [c for c in log.collected if c[0] == "STEPS"][-1][2]
        out[f"run{run}.steps"] = np.array(steps)
    out["mac_calls_t"] = np.array([c[0] for c in mac.calls])
    out["mac_calls_nbs"] = np.array([len(c[1]) for c in mac.calls])
    stepper.close_env()
    np.savez_compressed(os.path.join(OUT, "parallel_stepper.npz"), **out)


def _load_file_module(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def pfsp_fixture():
    pe = _load_file_module("ref_payoff_entry", os.path.join(REF_SRC, "league/components/payoff_entry.py"))
    sp = _load_file_module("ref_self_play", os.path.join(REF_SRC, "league/components/self_play.py"))
    rng = np.random.RandomState(11)
    n = 6
    payoff = th.zeros((n, n, 5))
    payoff[..., 0] = th.tensor(rng.randint(0, 6, size=(n, n)), dtype=th.float32)  # GAMES (some zero)
    payoff[..., 1] = th.floor(payoff[..., 0] * th.tensor(rng.rand(n, n), dtype=th.float32))  # WIN
    payoff[..., 3] = th.floor((payoff[..., 0] - payoff[..., 1]) * 0.5)  # DRAW
    payoff[..., 2] = payoff[..., 0] - payoff[..., 1] - payoff[..., 3]  # LOSS
    wrap = pe.PayoffWrapper(payoff.clone())
    out = {"payoff": payoff.numpy()}
    recorded = []
    orig_choice = sp.np.random.choice

    def rec_choice(a, p=None, **kw):
        recorded.append(np.asarray(p, dtype=np.float64))
        return orig_choice(a, p=p, **kw)

    sp.np.random.choice = rec_choice
    samp = sp.PFSPSampling()
    for i in range(n):
        wr = wrap.win_rates(i)
        out[f"win_rates{i}"] = wr.numpy().copy()
        out[f"win_rates_idx{i}"] = wrap.win_rates(i, [0, 2, 4]).numpy().copy()
        for w in ["linear", "squared", "variance", "linear_capped"]:
            recorded.clear()
            samp.sample(list(range(n)), prio_measure=wr, weighting=w)
            out[f"p{i}.{w}"] = recorded[0]
    sp.np.random.choice = orig_choice
    np.savez_compressed(os.path.join(OUT, "pfsp.npz"), **out)


def checkpoint_fixture():
    """Checkpoint interop (q_learner.py:133-147, basic_controller.py:68-72, run_utils.py:20-37).

    A reference QLearner (qmix, double-Q; the qlearner_qmix_dq setup) trains once and writes its checkpoint
    as ckpt_qmix/100/home_qlearner_{agent,mixer,opt}.th (the layout models/{token}/{t_env}/ the experiment
    saves). A FRESH reference learner (seed 99) then resumes from it (load_models) and trains once more.
    checkpoint.npz: the batch (b.*), the resumed learner's untouched target mixer (tm.*: load_models does
    not load it), the stats of the resumed call (stat.*) and all parameters after it (p2.*)."""
    import shutil
    th.manual_seed(7)
    args = base_args()
    B, T, N, d_obs, A, S = 4, 7, 5, 80, 15, 60
    batch, scheme, groups, preprocess = make_batch(B, T, N, d_obs, A, S, [6, 3, 4, 2], seed=8)
    mac = BasicMAC(batch.scheme, groups, args)
    learner = QLearner(mac, batch.scheme, StatLogger(), args, name="home")
    learner.build_optimizer()
    learner.train(batch, 100, 0)
    ck = os.path.join(OUT, "ckpt_qmix")
    shutil.rmtree(ck, ignore_errors=True)
    os.makedirs(os.path.join(ck, "100"))
    learner.save_models(os.path.join(ck, "100"), "home")

    th.manual_seed(99)
    mac2 = BasicMAC(batch.scheme, groups, args)
    logger2 = StatLogger()
    learner2 = QLearner(mac2, batch.scheme, logger2, args, name="home")
    learner2.build_optimizer()
    out = {}
    out.update(sd_to_np("tm.", learner2.target_mixer.state_dict()))
    learner2.load_models(os.path.join(ck, "100"))
    out.update(batch_to_np("b.", batch))
    learner2.train(batch, 200, 32)
    stats = {k.replace("home_qlearner_", ""): v for k, v, _ in logger2.stats}
    for k in ["loss", "grad_norm", "td_error_abs", "q_taken_mean", "target_mean"]:
        out[f"stat.{k}"] = np.array(stats[k], dtype=np.float64)
    out.update(sd_to_np("p2.agent.", mac2.agent.state_dict()))
    out.update(sd_to_np("p2.target_agent.", learner2.target_mac.agent.state_dict()))
    out.update(sd_to_np("p2.mixer.", learner2.mixer.state_dict()))
    np.savez_compressed(os.path.join(OUT, "checkpoint.npz"), **out)


def logger_fixture():
    """MainLogger collect/log/preprocess (custom_logging/logger.py:24-173, collectibles.py:10-68).

    Probe shims (this generator only): collections.Sized aliased (logger.py:3); custom_logging.platforms
    stubbed with inert classes (its tensorboard/sacred sinks need packages absent here) -- only the
    aggregation logic runs. Records a scripted sequence of collect()/log() calls (train interval, test
    completion) and the resulting stats: logger.npz keys `k{i}` (stat name), `t{i}`, `v{i}` (float64, NaN kept)."""
    collections.Sized = collections.abc.Sized
    plat = types.ModuleType("custom_logging.platforms")
    plat.CustomSacredLogger = plat.CustomTensorboardLogger = type("Inert", (), {})
    console = types.ModuleType("custom_logging.platforms.console")
    console.CustomConsoleLogger = type("InertConsole", (), {"info": lambda self, *a: None})
    sys.modules["custom_logging.platforms"] = plat
    sys.modules["custom_logging.platforms.console"] = console
    from custom_logging.logger import MainLogger
    from custom_logging.collectibles import Collectibles
    from custom_logging.utils.enums import Originator
    lg = MainLogger(console.CustomConsoleLogger(), SimpleNamespace(test_nepisode=4, runner_log_interval=100))

    def run(rets, won_h, won_a, draw, steps):
        lg.collect(Collectibles.RETURN, rets, origin=Originator.HOME, parallel=True)
        lg.collect(Collectibles.WON, won_h, origin=Originator.HOME, parallel=True)
        lg.collect(Collectibles.WON, won_a, origin=Originator.AWAY, parallel=True)
        lg.collect(Collectibles.DRAW, draw, parallel=True)
        lg.collect(Collectibles.STEPS, steps, parallel=True)  # an int with parallel=True: dropped (logger.py:135)

    run([1.5, 2.0, -1.0], [True, False, True], [False, True, False], [False, False, False], 37)
    lg.log(0)                       # first train log (log_train_stats_t starts at -1e6)
    run([0.25], [False], [False], [True], 12)
    lg.log(50)                      # inside the interval: nothing
    run([3.0, 4.5], [True, True], [False, False], [False, False], 20)
    lg.log(150)                     # logs both runs' data
    lg.collect(Collectibles.RETURN, 7.0, origin=Originator.HOME)  # non-parallel scalar append
    lg.collect(Collectibles.WON, True, origin=Originator.HOME)
    lg.collect(Collectibles.DRAW, False)
    lg.log(200)                     # interval not reached
    lg.test_mode = True
    run([1.0, 2.0], [True, False], [False, False], [False, True], 9)
    lg.log(260)                     # test not finished (2 of 4)
    run([5.0, 6.0], [False, False], [True, False], [False, False], 9)
    lg.log(260)                     # test finished: test_* stats
    lg.test_mode = False
    lg.log(270)                     # 120 since the last train log: logs the scalar collects above
    lg.log(351)                     # inside the interval again: nothing
    out, i = {}, 0
    for k in sorted(lg.stats):
        for t, v in lg.stats[k]:
            out[f"k{i}"], out[f"t{i}"] = np.array(k), np.array(t, dtype=np.int64)
            out[f"v{i}"] = np.array(np.nan if v is None else v, dtype=np.float64)
            i += 1
    out["n"] = np.array(i, dtype=np.int64)
    np.savez_compressed(os.path.join(OUT, "logger.npz"), **out)


def _all():
    drqn_fixture()
    mac_fixture()
    eps_fixture()
    qmix_fixture()
    qlearner_fixture("qmix_dq", True)
    qlearner_fixture("qmix_nodq", False, double_q=False)
    qlearner_fixture("vdn", False, mixer="vdn")
    replay_fixture()
    pfsp_fixture()


if __name__ == "__main__":
    if "--checkpoint-only" in sys.argv:
        checkpoint_fixture()
        sys.exit(0)
    if "--logger-only" in sys.argv:
        logger_fixture()
        sys.exit(0)
    if "--stepper-only" not in sys.argv:
        _all()
        checkpoint_fixture()
        logger_fixture()
    _stepper_fixture()
    print("golden fixtures written to", OUT)
