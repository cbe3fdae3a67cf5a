"""REFIL (config 5) host logic on CPU: entity env spec, config layering and experiment wiring (no kernel calls),
the C oracle's entity env invariants, the imagine-group mask algebra against the oracle, and the CPU baseline."""
import numpy as np
import pytest
import torch

import envref
import refil_ref as RR
from helpers import refil_args


def test_entity_env_spec_from_env_args():
    from maleague.envs import EntityEnvSpec
    s = EntityEnvSpec.from_env_args({"match_build_plan": "refil_8", "min_agents": 3, "max_agents": 8, "seed": 5})
    assert (s.S, s.U, s.n_agents, s.n_entities, s.n_actions) == (8, 16, 8, 16, 21)
    info = s.env_info()
    assert info["entity_shape"] == 8 and info["n_entities"] == 16 and info["episode_limit"] == 100
    c = s.to_c()
    assert c.base.U == 16 and c.base.n_agents == 8 and c.base.policy_team == 0
    assert list(c.base.scripted) == [0, 1] and (c.min_agents, c.max_agents) == (3, 8)
    assert [c.base.team[u] for u in range(16)] == [0] * 8 + [1] * 8
    assert [c.base.role[u] for u in range(8)] == [c.base.role[u + 8] for u in range(8)]
    with pytest.raises(ValueError):
        EntityEnvSpec.from_env_args({"min_agents": 5, "max_agents": 4})
    with pytest.raises(ValueError):
        EntityEnvSpec.from_env_args({"max_agents": 9})


def test_refil_config_layers_and_experiment_wiring():
    """algs/refil + envs/ma_entity resolve to the entity stepper, EntityMAC, REFILLearner and FlexQMixer; the
    learner's flat parameter order is the kernel's (checked without a GPU)."""
    from maleague.controllers import EntityMAC
    from maleague.custom_logging import MainLogger
    from maleague.learners import REFILLearner
    from maleague.runs import MultiAgentExperiment
    from maleague.steppers import EntityParallelStepper
    from maleague.utils.config import build_config, to_args
    cfg = build_config("refil", "ma_entity", overrides=["batch_size_run=4", "runner=parallel", "buffer_size=8",
                                                        "buffer_cpu_only=True", "env_args.episode_limit=10"],
                       cuda_available=False)
    a = to_args(cfg)
    assert a.entity_scheme and a.mac == "entity" and a.learner == "refil" and a.mixer == "flex_qmix"
    exp = MultiAgentExperiment(a, MainLogger(log_interval=10 ** 12))
    assert isinstance(exp.stepper, EntityParallelStepper)
    assert isinstance(exp.home_mac, EntityMAC) and isinstance(exp.home_learner, REFILLearner)
    assert set(exp.scheme) >= {"entities", "obs_mask", "entity_mask", "avail_actions", "actions", "reward"}
    assert exp.home_buffer.data.transition_data["entities"].shape == (8, 11, 16, 8)
    assert exp.args.n_entities == 16 and exp.args.entity_shape == 8
    n = sum(p.numel() for p in exp.home_learner.parameters())
    assert n == 130645 and exp.home_learner._flat.flat.numel() == n
    sd = exp.home_learner.mixer.state_dict()
    assert "hyper_w_1.attn.in_trans.weight" in sd and "V.fc2.bias" in sd and "hyper_b_1.attn.scale_factor" in sd


def test_entity_oracle_env_invariants():
    roles, melees = [0, 2, 1, 2, 0, 2, 1, 2], [0, 0, 0, 0, 1, 0, 0, 1]
    ks = set()
    for b in range(24):
        e = envref.RefEntityEnv(roles, melees, 3, 8, seed=2, env_index=b)
        e.reset()
        ks.add(e.k)
        ent, om, em = e.entities()
        k = e.k
        assert 3 <= k <= 8
        assert (em[:k] == 0).all() and (em[k:8] == 1).all() and (em[8:8 + k] == 0).all() and (em[8 + k:] == 1).all()
        assert (ent[em == 1] == 0).all() and (ent[em == 0, 0] == 1).all()
        assert all(om[i, i] == 0 for i in range(16) if em[i] == 0)
        assert (om[em == 1] == 1).all() and (om[:, em == 1] == 1).all()
        av = e.avail()
        assert (av[k:, 0] == 1).all() and (av[k:, 1:] == 0).all() and (av[:k, 0] == 0).all()
        # deterministic under the counter RNG
        e2 = envref.RefEntityEnv(roles, melees, 3, 8, seed=2, env_index=b)
        e2.reset()
        assert e2.k == k and np.array_equal(e2.entities()[0], ent)
    assert len(ks) >= 4


def test_imagine_masks_match_oracle():
    from maleague.modules.agents.entity_agent import imagine_masks
    g = torch.Generator().manual_seed(3)
    bs, ts, ne = 5, 4, 16
    em = (torch.rand(bs, ts, ne, generator=g) < 0.3).to(torch.uint8)
    om = (torch.rand(bs, ts, ne, ne, generator=g) < 0.4).to(torch.uint8)
    ga = (torch.rand(bs, 1, ne, generator=g) < 0.5).to(torch.uint8)
    got = imagine_masks(ga, em, om)
    want = RR.imagine_masks(ga, em, om)
    for x, y in zip(got, want):
        assert torch.equal(x.to(torch.uint8), y.to(torch.uint8))


def test_refil_cpu_baseline_runs():
    import cpu_baseline
    r = cpu_baseline.run_refil(seconds=0.5, B=4, episode_limit=10, threads=2, batch_size=4)
    assert r["env_steps"] > 0 and r["runs"] >= 1 and r["value"] > 0


def test_refil_args_helper_matches_fixture_dims():
    a = refil_args()
    assert a.entity_shape + a.n_actions == 29 and a.attn_embed_dim == 64 and a.attn_n_heads == 4
