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
