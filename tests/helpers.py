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
