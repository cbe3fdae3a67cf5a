"""Shared test helpers (args namespaces, spec <-> oracle env construction)."""
from types import SimpleNamespace

import numpy as np


def qmix_args(**kw):
    """Default + qmix.yaml + ma.yaml values that matter on the hot path (src/config/*.yaml)."""
    a = dict(n_agents=5, n_actions=15, state_shape=60, rnn_hidden_dim=64, obs_last_action=True, obs_agent_id=True,
             agent="rnn", agent_output_type="q", action_selector="epsilon_greedy", epsilon_start=1.0,
             epsilon_finish=0.05, epsilon_anneal_time=50000, freeze_native=False, device="cuda", mixer="qmix",
             mixing_embed_dim=32, hypernet_layers=2, hypernet_embed=64, double_q=True, gamma=0.99, lr=0.0005,
             optim_alpha=0.99, optim_eps=1e-5, grad_norm_clip=10, target_update_interval=200,
             learner_log_interval=0, batch_size_run=8, batch_size=32, buffer_size=64, seed=0,
             env_args={"match_build_plan": "medium_1h_4t", "grid_size": 20, "stochastic_spawns": True,
                       "episode_limit": 100})
    a.update(kw)
    return SimpleNamespace(**a)


def ref_envs_for(spec, B, seed=0):
    """oracle RefEnv instances matching a product TeamsEnvSpec (same unit tables, keys seed*2^32 + b)."""
    import envref
    return [envref.RefEnv(spec.team, spec.role, spec.melee, spec.scripted, grid=spec.grid,
                          episode_limit=spec.episode_limit, stochastic=spec.stochastic, seed=seed, env_index=b)
            for b in range(B)]


def scheme_for(env_info, torch):
    from maleague.components.transforms import OneHot
    scheme = {
        "state": {"vshape": env_info["state_shape"]},
        "obs": {"vshape": env_info["obs_shape"], "group": "agents"},
        "actions": {"vshape": (1,), "group": "agents", "dtype": torch.long},
        "avail_actions": {"vshape": (env_info["n_actions"],), "group": "agents", "dtype": torch.int},
        "reward": {"vshape": (1,)},
        "terminated": {"vshape": (1,), "dtype": torch.uint8},
    }
    groups = {"agents": env_info["n_agents"]}
    preprocess = {"actions": ("actions_onehot", [OneHot(out_dim=env_info["n_actions"])])}
    return scheme, groups, preprocess


def np_batch(batch):
    return {k: v.detach().cpu().numpy() for k, v in batch.data.transition_data.items()}


def refil_args(**kw):
    """REFIL (config 5) args: entity scheme + imagine agent + flex_qmix (REFIL defaults)."""
    a = dict(n_agents=8, n_entities=16, n_actions=21, entity_shape=8, entity_last_action=True, attn_embed_dim=64,
             attn_n_heads=4, rnn_hidden_dim=64, hypernet_embed=64, mixing_embed_dim=32, pooling_type=None,
             softmax_mixing_weights=False, mixer="flex_qmix", entity_scheme=True, agent="imagine_entity_attend_rnn",
             mac="entity", learner="refil", agent_output_type="q", action_selector="epsilon_greedy",
             epsilon_start=1.0, epsilon_finish=0.05, epsilon_anneal_time=50000, double_q=True, gamma=0.99, lr=5e-4,
             optim_alpha=0.99, optim_eps=1e-5, weight_decay=0, grad_norm_clip=10, target_update_interval=200,
             learner_log_interval=0, lmbda=0.5, device="cuda", freeze_native=False, obs_last_action=False,
             obs_agent_id=False, batch_size_run=8, batch_size=32, buffer_size=64, seed=0, runner="parallel",
             env_args={"match_build_plan": "refil_8", "grid_size": 20, "stochastic_spawns": True,
                       "episode_limit": 100, "min_agents": 3, "max_agents": 8})
    a.update(kw)
    return SimpleNamespace(**a)


def entity_scheme_for(env_info, torch):
    from maleague.components.transforms import OneHot
    NE, ED, A = env_info["n_entities"], env_info["entity_shape"], env_info["n_actions"]
    scheme = {
        "entities": {"vshape": (NE, ED)},
        "obs_mask": {"vshape": (NE, NE), "dtype": torch.uint8},
        "entity_mask": {"vshape": (NE,), "dtype": torch.uint8},
        "actions": {"vshape": (1,), "group": "agents", "dtype": torch.long},
        "avail_actions": {"vshape": (A,), "group": "agents", "dtype": torch.int},
        "reward": {"vshape": (1,)},
        "terminated": {"vshape": (1,), "dtype": torch.uint8},
    }
    groups = {"agents": env_info["n_agents"]}
    preprocess = {"actions": ("actions_onehot", [OneHot(out_dim=A)])}
    return scheme, groups, preprocess


def ref_entity_envs_for(spec, B, seed=0):
    import envref
    return [envref.RefEntityEnv(spec.roles, spec.melees, spec.min_agents, spec.max_agents, grid=spec.grid,
                                episode_limit=spec.episode_limit, stochastic=spec.stochastic, seed=seed, env_index=b)
            for b in range(B)]


def assert_near_tie_divergence(ref_sides, got_sides, q_sides, B, tol=1e-5):
    """two kernels that agree in fp32 up to summation order must produce the same episodes except where a
    near-tie flips an argmax. For every episode that differs (over every side of a self-play pair), the first differing
    step t must have identical pre-transition data (state, obs, avail, filled: the env states agree up to t) and differ
    in the actions, and each differing pick must be a near-tie of the fp32 oracle's Q along the recorded trajectory
    (|Q[a_got] - Q[a_ref]| <= tol, both available). Returns the number of differing episodes."""
    import numpy as np
    pre_keys = ("state", "obs", "avail_actions", "filled")
    n_diff = 0
    for b in range(B):
        t_first = None
        T1 = got_sides[0]["actions"].shape[1]
        for t in range(T1):
            if any(not np.array_equal(r[k][b, t], g[k][b, t]) for r, g in zip(ref_sides, got_sides) for k in g):
                t_first = t
                break
        if t_first is None:
            continue
        n_diff += 1
        flips = 0
        for r, g, q in zip(ref_sides, got_sides, q_sides):
            for k in pre_keys:
                if k in g:
                    assert np.array_equal(r[k][b, t_first], g[k][b, t_first]), (b, t_first, k)
            av = g["avail_actions"][b, t_first].astype(bool)
            for n in np.nonzero(r["actions"][b, t_first, :, 0] != g["actions"][b, t_first, :, 0])[0]:
                ag, ar = int(g["actions"][b, t_first, n, 0]), int(r["actions"][b, t_first, n, 0])
                assert av[n, ag] and av[n, ar], (b, t_first, n)
                assert abs(float(q[b, t_first, n, ag]) - float(q[b, t_first, n, ar])) <= tol, (b, t_first, n, ag, ar)
                flips += 1
        assert flips > 0, f"episode {b} diverges at t={t_first} without an action flip"
    return n_diff
