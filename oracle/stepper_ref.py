"""CPU restatement of ParallelStepper.run bookkeeping (src/steppers/parallel_stepper.py:82-216).

TEST INFRASTRUCTURE ONLY. Pinned against tests/golden/parallel_stepper.npz, captured from the
reference stepper itself with a scripted fake env. Restated semantics:
  * reset: pre-transition data (state, avail, obs) at t=0, filled[:, 0] = 1            (:82-104)
  * per iteration t: actions for `running` envs recorded at t (mark_filled=False)       (:132-141)
  * step every not-yet-terminated env; `running` recomputed BEFORE receiving, so an env
    that terminates at t is still in `running` at t+1 and gets (and records) an action  (:143-155)
  * receive: reward[0], terminated=any(done_n), env_info kept on termination, next
    pre-transition data written at t+1 with filled=1                                     (:168-200)
  * t_env += one per received step in train mode; self.t = iterations that received      (:178-179,197,202-203)
Envs are adapters: reset(i) -> (state, avail, obs); step(i, actions) ->
(reward_list, done_bool, info, state, avail, obs). policy(t, env_ids, batch) -> actions [len, N].
"""
from __future__ import annotations

import numpy as np


def new_batch(B, T1, N, A, d_obs, S):
    return {"state": np.zeros((B, T1, S), np.float32), "obs": np.zeros((B, T1, N, d_obs), np.float32),
            "actions": np.zeros((B, T1, N, 1), np.int64), "avail_actions": np.zeros((B, T1, N, A), np.int32),
            "reward": np.zeros((B, T1, 1), np.float32), "terminated": np.zeros((B, T1, 1), np.uint8),
            "actions_onehot": np.zeros((B, T1, N, A), np.float32), "filled": np.zeros((B, T1, 1), np.int64)}


def run(envs, policy, B, T1, N, A, d_obs, S, test_mode=False):
    batch = new_batch(B, T1, N, A, d_obs, S)
    for i in range(B):
        st, av, ob = envs.reset(i)
        batch["state"][i, 0], batch["avail_actions"][i, 0], batch["obs"][i, 0] = st, av, ob
        batch["filled"][i, 0] = 1
    terminated = [False] * B
    running = list(range(B))
    returns = [0.0] * B
    env_infos, info_env = [], []
    steps_this_run = 0
    t = 0
    while True:
        acts = np.asarray(policy(t, list(running), batch), dtype=np.int64).reshape(len(running), N)
        for k, i in enumerate(running):
            batch["actions"][i, t, :, 0] = acts[k]
            batch["actions_onehot"][i, t] = 0
            batch["actions_onehot"][i, t, np.arange(N), acts[k]] = 1.0
        sent = {i: acts[k] for k, i in enumerate(running) if not terminated[i]}
        running = [i for i in range(B) if not terminated[i]]
        if all(terminated):
            break
        for i in range(B):
            if terminated[i]:
                continue
            rew, done, info, st, av, ob = envs.step(i, sent[i])
            r0 = rew[0]
            returns[i] += r0
            if not test_mode:
                steps_this_run += 1
            if done:
                env_infos.append(info)
                info_env.append(i)
            terminated[i] = done
            batch["reward"][i, t, 0] = r0
            batch["terminated"][i, t, 0] = done
            batch["state"][i, t + 1], batch["avail_actions"][i, t + 1], batch["obs"][i, t + 1] = st, av, ob
            batch["filled"][i, t + 1] = 1
        t += 1
    return {"batch": batch, "t": t, "env_steps": steps_this_run, "returns": returns, "env_infos": env_infos,
            "info_env": info_env}


def run_self_play(envs, home_policy, away_policy, B, T1, N, A, d_obs, S, test_mode=False):
    """SelfPlayParallelStepper.run bookkeeping (src/steppers/self_play_parallel_stepper.py:50-201, intended
    semantics: the reference's .send/.recv on Queues is defect SURVEY App. A). Same loop as run(); the env
    gets cat(home, away) actions (:108), obs / avail are split home = first N agents, away = the rest, state
    goes to both (stepper_utils.py:4-24), reward (home, away) = reward[0], reward[1] (:159)."""
    home, away = new_batch(B, T1, N, A, d_obs, S), new_batch(B, T1, N, A, d_obs, S)

    def pre(i, t, st, av, ob):
        for b, sl in ((home, slice(0, N)), (away, slice(N, 2 * N))):
            b["state"][i, t], b["avail_actions"][i, t], b["obs"][i, t] = st, av[sl], ob[sl]
            b["filled"][i, t] = 1

    for i in range(B):
        pre(i, 0, *envs.reset(i))
    terminated = [False] * B
    running = list(range(B))
    returns = [[0.0] * B, [0.0] * B]
    env_infos, info_env = [], []
    steps_this_run = 0
    t = 0
    while True:
        ah = np.asarray(home_policy(t, list(running), home), dtype=np.int64).reshape(len(running), N)
        aa = np.asarray(away_policy(t, list(running), away), dtype=np.int64).reshape(len(running), N)
        for b, acts in ((home, ah), (away, aa)):
            for k, i in enumerate(running):
                b["actions"][i, t, :, 0] = acts[k]
                b["actions_onehot"][i, t] = 0
                b["actions_onehot"][i, t, np.arange(N), acts[k]] = 1.0
        sent = {i: np.concatenate([ah[k], aa[k]]) for k, i in enumerate(running) if not terminated[i]}
        running = [i for i in range(B) if not terminated[i]]
        if all(terminated):
            break
        for i in range(B):
            if terminated[i]:
                continue
            rew, done, info, st, av, ob = envs.step(i, sent[i])
            for side, b in enumerate((home, away)):
                returns[side][i] += rew[side]
                b["reward"][i, t, 0] = rew[side]
                b["terminated"][i, t, 0] = done
            if not test_mode:
                steps_this_run += 1
            if done:
                env_infos.append(info)
                info_env.append(i)
            terminated[i] = done
            pre(i, t + 1, st, av, ob)
        t += 1
    return {"home": home, "away": away, "t": t, "env_steps": steps_this_run, "returns": returns,
            "env_infos": env_infos, "info_env": info_env}


class RefVecEnv:
    """Adapter over oracle/envref.RefEnv instances for run()."""

    def __init__(self, envs):
        self.envs = envs

    def reset(self, i):
        e = self.envs[i]
        e.reset()
        return e.state(), e.avail(), e.obs()

    def step(self, i, actions):
        e = self.envs[i]
        rew, done, info = e.step(actions)
        return rew, done, info, e.state(), e.avail(), e.obs()
