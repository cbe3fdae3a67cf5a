"""YAML config layering (behaviour of src/utils/config_builder.py:19-62 and main_utils.py:33-126).

Precedence, low to high: default < envs/<env> < leagues/<league> < algs/<alg> < overrides. With a
``config_dir`` (e.g. the reference's own src/config) the YAML files there are read unchanged; without
one, the built-in defaults below (the hot-path keys of default.yaml / algs/qmix.yaml / envs/ma.yaml)
are used. Overrides accept ``key=value`` / ``--key=value`` / ``--env_args.key=value`` and, unlike the
reference (main_utils.py:118-126), also string values (values are parsed with yaml.safe_load).
"""
from __future__ import annotations

import copy
import os
from collections.abc import Mapping
from types import SimpleNamespace

import yaml

BUILTIN = {
    "default": {
        "runner": "episode", "mac": "basic", "env": "ma", "env_args": {}, "batch_size_run": 1, "test_nepisode": 20,
        "test_interval": 2000, "test_greedy": True, "log_interval": 2000, "runner_log_interval": 2000,
        "learner_log_interval": 2000, "t_max": 10000, "use_cuda": True, "buffer_cpu_only": True,
        "use_tensorboard": False, "save_model": False, "save_model_interval": 2000000, "checkpoint_path": "",
        "evaluate": False, "load_step": 0, "save_replay": False, "local_results_path": "results", "gamma": 0.99,
        "batch_size": 32, "buffer_size": 32, "lr": 0.0005, "critic_lr": 0.0005, "optim_alpha": 0.99,
        "optim_eps": 0.00001, "grad_norm_clip": 10, "agent": "rnn", "rnn_hidden_dim": 64, "obs_agent_id": True,
        "obs_last_action": True, "repeat_id": 1, "label": "default_label", "freeze_native": False, "sfs": None,
        "headless_controls": True,
    },
    "envs/ma": {
        "env": "ma", "play_mode": "normal",
        "env_args": {"headless": True, "record": False, "fps": 30, "draw_grid": False, "infos": False,
                     "global_reward": True, "grid_size": 20, "match_build_plan": "medium_1h_4t", "ai": "basic",
                     "stochastic_spawns": True, "attack_ranges_only": False},
        "test_greedy": True, "test_nepisode": 32, "test_interval": 10000, "log_interval": 10000,
        "runner_log_interval": 10000, "learner_log_interval": 10000, "t_max": 2050000, "show_exp_parameters": True,
    },
    "algs/qmix": {
        "action_selector": "epsilon_greedy", "epsilon_start": 1.0, "epsilon_finish": 0.05,
        "epsilon_anneal_time": 50000, "runner": "episode", "buffer_size": 5000, "target_update_interval": 200,
        "agent_output_type": "q", "learner": "q", "double_q": True, "mixer": "qmix", "mixing_embed_dim": 32,
        "hypernet_layers": 2, "hypernet_embed": 64, "name": "qmix",
    },
    # REFIL (config 5): the reference vendors the modules without a config; these are the values of
    # the golden fixtures (tests/golden/make_refil_golden.py) with the qmix.yaml schedule / buffer.
    "algs/refil": {
        "action_selector": "epsilon_greedy", "epsilon_start": 1.0, "epsilon_finish": 0.05,
        "epsilon_anneal_time": 50000, "runner": "episode", "buffer_size": 5000, "target_update_interval": 200,
        "agent_output_type": "q", "learner": "refil", "double_q": True, "mixer": "flex_qmix", "mixing_embed_dim": 32,
        "hypernet_embed": 64, "agent": "imagine_entity_attend_rnn", "mac": "entity", "attn_embed_dim": 64,
        "attn_n_heads": 4, "pooling_type": None, "softmax_mixing_weights": False, "lmbda": 0.5,
        "entity_last_action": True, "weight_decay": 0, "name": "refil",
    },
    "envs/ma_entity": {
        "env": "ma_entity", "entity_scheme": True,
        "env_args": {"grid_size": 20, "match_build_plan": "refil_8", "ai": "basic", "stochastic_spawns": True,
                     "min_agents": 3, "max_agents": 8, "episode_limit": 100},
        "test_greedy": True, "test_nepisode": 32, "test_interval": 10000, "log_interval": 10000,
        "runner_log_interval": 10000, "learner_log_interval": 10000, "t_max": 2050000, "show_exp_parameters": True,
    },
    # src/config/leagues/matchmaking.yaml (the league layer: per-match play time, league run time, matchmaking)
    "leagues/matchmaking": {
        "play_time_mins": 120, "league_runtime_hours": 24, "n_league_evaluation_episodes": 100,
        "show_exp_parameters": True, "buffer_cpu_only": False, "mac": "basic", "headless_controls": False,
        "use_cuda": True, "use_tensorboard": True, "matchmaking": "pfsp",
    },
    # src/config/leagues/test.yaml (a short league: 1-minute matches, 6 minutes in all)
    "leagues/test": {
        "team_size": 5, "play_time_mins": 1, "league_runtime_hours": 0.1, "n_league_evaluation_episodes": 1,
        "show_exp_parameters": True, "env_args": {"record": False, "fps": 60}, "buffer_cpu_only": True,
        "mac": "basic", "headless_controls": False, "use_cuda": True, "use_tensorboard": True, "matchmaking": "pfsp",
    },
    "algs/vdn": {
        "action_selector": "epsilon_greedy", "epsilon_start": 1.0, "epsilon_finish": 0.05,
        "epsilon_anneal_time": 50000, "runner": "episode", "buffer_size": 5000, "target_update_interval": 200,
        "agent_output_type": "q", "learner": "q", "double_q": True, "mixer": "vdn", "name": "vdn",
    },
}


def recursive_dict_update(dest, src):
    if not src:
        return dest
    for k, v in src.items():
        if isinstance(v, Mapping):
            dest[k] = recursive_dict_update(dict(dest.get(k, {}) or {}), v)
        else:
            dest[k] = v
    return dest


def _layer(config_dir, sub):
    if config_dir is not None:
        path = os.path.join(config_dir, f"{sub}.yaml")
        if os.path.exists(path):
            with open(path) as f:
                return yaml.safe_load(f) or {}
    return copy.deepcopy(BUILTIN.get(sub, {}))


def parse_override(token: str):
    tok = token[2:] if token.startswith("--") else token
    if "=" not in tok:
        raise ValueError(f"override {token!r} must look like key=value")
    key, raw = tok.split("=", 1)
    try:
        val = yaml.safe_load(raw)
    except yaml.YAMLError:
        val = raw
    return key, val


def apply_override(cfg: dict, key: str, val):
    parts = key.split(".")
    node = cfg
    for p in parts[:-1]:
        node = node.setdefault(p, {})
    node[parts[-1]] = val


def sanity_check(cfg: dict, cuda_available: bool | None = None) -> dict:
    """src/utils/run_utils.py:6-17."""
    if cuda_available is None:
        import torch
        cuda_available = torch.cuda.is_available()
    if cfg.get("use_cuda") and not cuda_available:
        cfg["use_cuda"] = False
    if cfg["test_nepisode"] < cfg["batch_size_run"]:
        cfg["test_nepisode"] = cfg["batch_size_run"]
    else:
        cfg["test_nepisode"] = (cfg["test_nepisode"] // cfg["batch_size_run"]) * cfg["batch_size_run"]
    return cfg


def build_config(alg="qmix", env="ma", league=None, overrides=(), config_dir=None, device_index=0,
                 cuda_available=None) -> dict:
    cfg = _layer(config_dir, "default")
    cfg = recursive_dict_update(cfg, _layer(config_dir, f"envs/{env}"))
    if league:
        cfg = recursive_dict_update(cfg, _layer(config_dir, f"leagues/{league}"))
    cfg = recursive_dict_update(cfg, _layer(config_dir, f"algs/{alg}"))
    for tok in overrides:
        apply_override(cfg, *parse_override(tok))
    cfg = sanity_check(cfg, cuda_available)
    cfg["device"] = f"cuda:{device_index}" if cfg.get("use_cuda") else "cpu"
    cfg["config_dir"] = config_dir
    return cfg


def to_args(cfg: dict) -> SimpleNamespace:
    return SimpleNamespace(**copy.deepcopy(cfg))
