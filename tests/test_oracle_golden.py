"""The CPU oracle (oracle/learner_ref.py, oracle/stepper_ref.py) against golden vectors produced by the
reference itself (tests/golden/make_golden.py). Runs on CPU."""
from types import SimpleNamespace

import numpy as np
import torch

import learner_ref as LR
import stepper_ref as SR

torch.set_num_threads(1)


def agent_params(d, prefix):
    return {k[len(prefix):]: torch.from_numpy(np.array(d[k])) for k in d.files if k.startswith(prefix)}


def args(**kw):
    a = dict(n_agents=5, n_actions=15, state_shape=60, rnn_hidden_dim=64, obs_last_action=True, obs_agent_id=True,
             mixer="qmix", mixing_embed_dim=32, hypernet_layers=2, hypernet_embed=64, double_q=True, gamma=0.99,
             lr=0.0005, optim_alpha=0.99, optim_eps=1e-5, grad_norm_clip=10, target_update_interval=200)
    a.update(kw)
    return SimpleNamespace(**a)


def test_drqn_step(golden):
    d = golden("drqn_step.npz")
    p = agent_params(d, "p.")
    q, h = LR.drqn_forward(p, torch.from_numpy(d["inputs"]), torch.from_numpy(d["hidden"]))
    np.testing.assert_allclose(q.numpy(), d["q"], atol=1e-5, rtol=1e-5)
    np.testing.assert_allclose(h.numpy(), d["h"], atol=1e-5, rtol=1e-5)


def test_mac_forward(golden):
    d = golden("mac_forward.npz")
    p = agent_params(d, "p.")
    b = LR.batch_from_npz(d)
    q, _ = LR.mac_unroll(p, b, 5)
    np.testing.assert_allclose(q.numpy(), np.transpose(d["q"], (1, 0, 2, 3)), atol=1e-5, rtol=1e-5)


def test_greedy_select(golden):
    d = golden("eps_greedy.npz")
    a = LR.greedy_select(torch.from_numpy(d["q"]), torch.from_numpy(d["avail"]))
    np.testing.assert_array_equal(a.numpy(), d["actions"])
    assert (d["is_greedy"] == 1).all()


def test_epsilon_schedule(golden):
    d = golden("eps_greedy.npz")
    lin = lambda t: max(0.05, 1.0 - (1.0 - 0.05) / 50000 * t)  # noqa: E731
    np.testing.assert_allclose([lin(int(t)) for t in d["sched_t"]], d["sched_eps"], rtol=0, atol=0)


def test_qmix_forward(golden):
    d = golden("qmix_fwd.npz")
    mp = agent_params(d, "p.")
    y = LR.qmix_forward(mp, torch.from_numpy(d["agent_qs"]), torch.from_numpy(d["states"]), 5, 32, 2)
    np.testing.assert_allclose(y.numpy(), d["q_tot"], atol=1e-5, rtol=1e-5)


def _run_learner(d, a, mixer_prefix):
    mp = agent_params(d, "p0.mixer.") if mixer_prefix else None
    ref = LR.QLearnerRef(agent_params(d, "p0.agent."), mp, a)
    out = []
    for i, (t_env, ep) in enumerate(d["calls"]):
        b = LR.batch_from_npz(d)
        out.append(ref.train(b, int(t_env), int(ep)))
    return ref, out


def _check_learner(name, a, mixer, golden, full):
    d = golden(name)
    ref, stats = _run_learner(d, a, mixer)
    for i, s in enumerate(stats):
        for k in ["loss", "grad_norm", "td_error_abs", "q_taken_mean", "target_mean"]:
            np.testing.assert_allclose(s[k], float(d[f"stat{i}.{k}"]), rtol=2e-5, atol=1e-6, err_msg=f"{k}@{i}")
    last = len(stats)
    st = ref.agent_state()
    for k, v in st.items():
        np.testing.assert_allclose(v.numpy(), d[f"p{last}.agent.{k}"], atol=2e-6, rtol=1e-5, err_msg=k)
    if mixer:
        for k, v in ref.mixer_state().items():
            np.testing.assert_allclose(v.numpy(), d[f"p{last}.mixer.{k}"], atol=2e-6, rtol=1e-5, err_msg=k)
    # target network was refreshed at the 3rd call (episode 232 - 0 >= 200)
    for k, v in ref.tp.items():
        np.testing.assert_allclose(v.numpy(), d[f"p{last}.target_agent.{k}"], atol=2e-6, rtol=1e-5)
    assert ref.trained_steps == int(d["trained_steps"])


def test_qlearner_qmix_double_q(golden):
    _check_learner("qlearner_qmix_dq.npz", args(), True, golden, True)


def test_qlearner_qmix_single_q(golden):
    _check_learner("qlearner_qmix_nodq.npz", args(double_q=False), True, golden, False)


def test_qlearner_vdn(golden):
    _check_learner("qlearner_vdn.npz", args(mixer="vdn"), False, golden, False)


def test_pfsp_weightings(golden):
    d = golden("pfsp.npz")
    payoff = d["payoff"]
    n = payoff.shape[0]
    for i in range(n):
        games = payoff[i, :, 0]
        with np.errstate(divide="ignore", invalid="ignore"):
            wr = (payoff[i, :, 1] + 0.5 * payoff[i, :, 3]) / games
        wr[games == 0] = 0.5
        np.testing.assert_allclose(wr, d[f"win_rates{i}"], rtol=1e-6)
        fns = {"linear": lambda x: 1 - x, "squared": lambda x: (1 - x) ** 2, "variance": lambda x: x * (1 - x),
               "linear_capped": lambda x: np.minimum(0.5, 1 - x)}
        for w, fn in fns.items():
            p = fn(np.asarray(d[f"win_rates{i}"]))
            np.testing.assert_allclose(p / p.sum(), d[f"p{i}.{w}"], rtol=1e-6)


class FakeEnvs:
    """Same scripted fake env as tests/golden/make_golden.py::_stepper_fixture."""

    def __init__(self, term_at, N, A, d_obs, S):
        self.term_at, self.N, self.A, self.d_obs, self.S = term_at, N, A, d_obs, S
        self.t = [0] * len(term_at)

    def _pre(self, i):
        t = self.t[i]
        obs = [[i * 100 + t * 10 + n + 0.25 * k for k in range(self.d_obs)] for n in range(self.N)]
        st = [i * 1000 + t * 10 + k for k in range(self.S)]
        av = [[1 if (a + n + t + i) % 3 != 0 or a == 0 else 0 for a in range(self.A)] for n in range(self.N)]
        return np.array(st, np.float32), np.array(av, np.int32), np.array(obs, np.float32)

    def reset(self, i):
        self.t[i] = 0
        return self._pre(i)

    def step(self, i, actions):
        r = float(i) + 0.5 * self.t[i] + 0.01 * sum(int(a) for a in actions)
        done = self.t[i] == self.term_at[i]
        self.t[i] += 1
        info = {"battle_won": [i % 2 == 0, False], "draw": i == 3}
        st, av, ob = self._pre(i)
        return [r, -r], done, info, st, av, ob


def test_parallel_stepper_bookkeeping(golden):
    d = golden("parallel_stepper.npz")
    N, A, d_obs, S, B = 3, 6, 4, 5, 5
    term_at = [int(x) for x in d["term_at"]]
    envs = FakeEnvs(term_at, N, A, d_obs, S)

    def policy(t, ids, batch):
        out = []
        for e in ids:
            row = []
            for n in range(N):
                a = (t * 7 + e * 3 + n) % A
                while batch["avail_actions"][e, t, n, a] == 0:
                    a = (a + 1) % A
                row.append(a)
            out.append(row)
        return out

    t_env = 0
    for run in range(2):
        res = SR.run(envs, policy, B, 9, N, A, d_obs, S, test_mode=(run == 1))
        for k, v in res["batch"].items():
            np.testing.assert_allclose(v, d[f"run{run}.{k}"], err_msg=f"run{run}.{k}", rtol=0, atol=0)
        if run == 0:
            t_env += res["env_steps"]
        assert t_env == int(d[f"run{run}.t_env"])
        assert res["t"] == int(d[f"run{run}.t"]) == int(d[f"run{run}.steps"])
        np.testing.assert_allclose(res["returns"], d[f"run{run}.returns"], rtol=1e-12)
        assert [i["battle_won"][0] for i in res["env_infos"]] == list(d[f"run{run}.info_won0"])
        assert [i["draw"] for i in res["env_infos"]] == list(d[f"run{run}.info_draw"])
