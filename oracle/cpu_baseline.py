"""CPU baseline for bench.py (TEST INFRASTRUCTURE / BASELINE ONLY -- never the measured product).

The reference's hot path restated on the host: the ParallelStepper bookkeeping (stepper_ref.run), the
synthetic env in C (env_ref.c via ctypes, one call per env per step like EnvWorker), the DRQN agent
forward batched over all B*N rows per step in PyTorch-CPU (basic_controller.py:38-50), epsilon-greedy,
and one QLearner.train (learner_ref.QLearnerRef, PyTorch-CPU autograd + RMSprop) on 32 sampled episodes
per run -- the loop shape of ma_experiment.py:224-241. Runs for a bounded wall-clock sample.

Legs (bench.py runs this file as a child process that never touches the GPU, ``--json``):
  vector   run():               one process, the B envs stepped in a loop, the agent batched over B*N rows
  process  run_process_model(): the reference's process model (parallel_stepper.py:32-39,
           env_worker_process.py:27-71): B = host cores env-worker processes, one env each, a
           ("step", actions) / result-dict round trip per env per step over a pipe, the parent batching the
           agent forward over the B*N rows and training once per run
  refil    run_refil():         config 5 on the host
"""
from __future__ import annotations

import json
import multiprocessing as mp
import os
import platform
import sys
import time
from types import SimpleNamespace

import numpy as np
import torch

import envref
import learner_ref as LR
import stepper_ref as SR

PLAN_MEDIUM_1H_4T = {"team": [0] * 5 + [1] * 5, "role": [0, 0, 1, 0, 0] * 2, "melee": [0] * 10,
                     "scripted": [True, False]}


def _init_params(d_in, H, A, N, S, E=32, HE=64, seed=0):
    torch.manual_seed(seed)
    fc1, gru, fc2 = torch.nn.Linear(d_in, H), torch.nn.GRUCell(H, H), torch.nn.Linear(H, A)
    agent = {"fc1.weight": fc1.weight, "fc1.bias": fc1.bias, "gru.weight_ih": gru.weight_ih,
             "gru.weight_hh": gru.weight_hh, "gru.bias_ih": gru.bias_ih, "gru.bias_hh": gru.bias_hh,
             "fc2.weight": fc2.weight, "fc2.bias": fc2.bias}
    mix = {}
    for name, shapes in [("hyper_w_1", [(HE, S), (N * E, HE)]), ("hyper_w_final", [(HE, S), (E, HE)])]:
        l0, l2 = torch.nn.Linear(shapes[0][1], shapes[0][0]), torch.nn.Linear(shapes[1][1], shapes[1][0])
        mix.update({f"{name}.0.weight": l0.weight, f"{name}.0.bias": l0.bias, f"{name}.2.weight": l2.weight,
                    f"{name}.2.bias": l2.bias})
    hb, v0, v2 = torch.nn.Linear(S, E), torch.nn.Linear(S, E), torch.nn.Linear(E, 1)
    mix.update({"hyper_b_1.weight": hb.weight, "hyper_b_1.bias": hb.bias, "V.0.weight": v0.weight,
                "V.0.bias": v0.bias, "V.2.weight": v2.weight, "V.2.bias": v2.bias})
    det = lambda d: {k: v.detach().numpy().copy() for k, v in d.items()}  # noqa: E731
    return det(agent), det(mix)


def run(seconds=15.0, B=64, episode_limit=100, eps=0.05, threads=None, seed=0, batch_size=32, capacity=512):
    threads = threads or os.cpu_count()
    torch.set_num_threads(threads)
    p = PLAN_MEDIUM_1H_4T
    U, N = 10, 5
    A, d_obs, S = 5 + U, 8 * U, 6 * U
    d_in = d_obs + A + N
    agent, mix = _init_params(d_in, 64, A, N, S, seed=seed)
    args = SimpleNamespace(n_agents=N, n_actions=A, mixer="qmix", mixing_embed_dim=32, hypernet_layers=2,
                           double_q=True, gamma=0.99, lr=5e-4, optim_alpha=0.99, optim_eps=1e-5, grad_norm_clip=10,
                           target_update_interval=200, obs_last_action=True, obs_agent_id=True)
    learner = LR.QLearnerRef(agent, mix, args)
    envs = SR.RefVecEnv([envref.RefEnv(p["team"], p["role"], p["melee"], p["scripted"], episode_limit=episode_limit,
                                       seed=seed, env_index=b) for b in range(B)])
    T1 = episode_limit + 1
    eye = torch.eye(N).unsqueeze(0).expand(B, -1, -1).reshape(B * N, N)
    buffer, rng = [], np.random.RandomState(seed)
    env_steps, runs, trains = 0, 0, 0
    t_start = time.perf_counter()
    while time.perf_counter() - t_start < seconds:
        h = [torch.zeros(B * N, 64)]

        def policy(t, ids, batch):
            obs = torch.from_numpy(batch["obs"][:, t].reshape(B * N, d_obs))
            last = torch.from_numpy(batch["actions_onehot"][:, t - 1].reshape(B * N, A)) if t > 0 \
                else torch.zeros(B * N, A)
            with torch.no_grad():
                q, h[0] = LR.drqn_forward(learner.p, torch.cat([obs, last, eye], 1), h[0])
            q = q.view(B, N, A)[ids]
            av = torch.from_numpy(batch["avail_actions"][ids, t])
            a = LR.greedy_select(q, av).numpy()
            coin = rng.rand(*a.shape) < eps
            for (k, n) in zip(*np.nonzero(coin)):
                a[k, n] = rng.choice(np.nonzero(av[k, n].numpy())[0])
            return a

        res = SR.run(envs, policy, B, T1, N, A, d_obs, S)
        env_steps += res["env_steps"]
        runs += 1
        for b in range(B):
            buffer.append({k: v[b] for k, v in res["batch"].items()})
        del buffer[:-capacity]
        if len(buffer) >= batch_size:
            idx = rng.choice(len(buffer), batch_size, replace=False)
            smp = {k: torch.from_numpy(np.stack([buffer[i][k] for i in idx])) for k in buffer[0]}
            T = int(smp["filled"].sum(1).max())
            smp = {k: v[:, :T].clone() for k, v in smp.items()}
            learner.train(smp, env_steps, runs * B)
            trains += 1
    elapsed = time.perf_counter() - t_start
    return {"value": env_steps / elapsed, "env_steps": env_steps, "seconds": elapsed, "runs": runs, "trains": trains,
            "cores": threads, "B": B}


def run_refil(seconds=15.0, B=32, episode_limit=100, eps=0.05, threads=None, seed=0, batch_size=32, capacity=256):
    """Config 5 on the host: the entity env in C (env_ref.c entity variant, one call per env per step), the
    EntityAttentionRNNAgent step batched over B envs in PyTorch-CPU (refil_ref.entity_agent), epsilon-greedy, the
    ParallelStepper bookkeeping, and one REFILLearner.train (refil_ref.REFILLearnerRef) per run."""
    import refil_ref as RR
    threads = threads or os.cpu_count()
    torch.set_num_threads(threads)
    roles, melees = [0, 2, 1, 2, 0, 2, 1, 2], [0, 0, 0, 0, 1, 0, 0, 1]
    NA, NE, ED = 8, 16, 8
    A = 5 + NE
    args = SimpleNamespace(n_agents=NA, n_entities=NE, n_actions=A, entity_shape=ED, attn_embed_dim=64,
                           attn_n_heads=4, rnn_hidden_dim=64, hypernet_embed=64, mixing_embed_dim=32,
                           softmax_mixing_weights=False, double_q=True, gamma=0.99, lr=5e-4, optim_alpha=0.99,
                           optim_eps=1e-5, weight_decay=0, grad_norm_clip=10, target_update_interval=200, lmbda=0.5)
    torch.manual_seed(seed)

    def lin(o, i, bias=True):
        m = torch.nn.Linear(i, o, bias=bias)
        return m.weight.detach().clone(), (m.bias.detach().clone() if bias else None)

    D0 = ED + A
    ap = {}
    ap["fc1.weight"], ap["fc1.bias"] = lin(64, D0)
    ap["attn.in_trans.weight"], _ = lin(192, 64, False)
    ap["attn.out_trans.weight"], ap["attn.out_trans.bias"] = lin(64, 64)
    ap["fc2.weight"], ap["fc2.bias"] = lin(64, 64)
    g = torch.nn.GRUCell(64, 64)
    ap.update({"rnn.weight_ih": g.weight_ih.detach(), "rnn.weight_hh": g.weight_hh.detach(),
               "rnn.bias_ih": g.bias_ih.detach(), "rnn.bias_hh": g.bias_hh.detach()})
    ap["fc3.weight"], ap["fc3.bias"] = lin(A, 64)
    mp = {}
    for h in ("hyper_w_1", "hyper_w_final", "hyper_b_1", "V"):
        mp[f"{h}.fc1.weight"], mp[f"{h}.fc1.bias"] = lin(64, D0)
        mp[f"{h}.attn.in_trans.weight"], _ = lin(192, 64, False)
        mp[f"{h}.attn.out_trans.weight"], mp[f"{h}.attn.out_trans.bias"] = lin(64, 64)
        mp[f"{h}.fc2.weight"], mp[f"{h}.fc2.bias"] = lin(32, 64)
    learner = RR.REFILLearnerRef(ap, mp, args)
    envs = [envref.RefEntityEnv(roles, melees, 3, 8, episode_limit=episode_limit, seed=seed, env_index=b)
            for b in range(B)]
    T1 = episode_limit + 1
    rng = np.random.RandomState(seed)
    buffer = []
    env_steps, runs, trains = 0, 0, 0
    t_start = time.perf_counter()
    while time.perf_counter() - t_start < seconds:
        bt = {"entities": np.zeros((B, T1, NE, ED), np.float32), "obs_mask": np.zeros((B, T1, NE, NE), np.uint8),
              "entity_mask": np.zeros((B, T1, NE), np.uint8), "actions": np.zeros((B, T1, NA, 1), np.int64),
              "avail_actions": np.zeros((B, T1, NA, A), np.int32), "reward": np.zeros((B, T1, 1), np.float32),
              "terminated": np.zeros((B, T1, 1), np.uint8), "actions_onehot": np.zeros((B, T1, NA, A), np.float32),
              "filled": np.zeros((B, T1, 1), np.int64)}

        def observe(b, t):
            bt["entities"][b, t], bt["obs_mask"][b, t], bt["entity_mask"][b, t] = envs[b].entities()
            bt["avail_actions"][b, t] = envs[b].avail()
            bt["filled"][b, t] = 1

        for b in range(B):
            envs[b].reset()
            observe(b, 0)
        status = np.zeros(B, np.int32)  # 0 running, 1 final action pending, 2 done
        h = torch.zeros(B, NA, 64)
        t = 0
        while (status < 2).any():
            ent = torch.from_numpy(bt["entities"][:, t])
            la = torch.zeros(B, NE, A)
            if t > 0:
                la[:, :NA] = torch.from_numpy(bt["actions_onehot"][:, t - 1])
            with torch.no_grad():
                q, hs = RR.entity_agent(learner.agent, torch.cat([ent, la], 2).unsqueeze(1),
                                        torch.from_numpy(bt["obs_mask"][:, t]).unsqueeze(1),
                                        torch.from_numpy(bt["entity_mask"][:, t]).unsqueeze(1), h, args)
            h = hs[:, 0]
            av = bt["avail_actions"][:, t]
            qm = np.where(av != 0, q[:, 0].numpy(), -np.inf)
            acts = qm.argmax(-1)
            coin = rng.rand(B, NA) < eps
            for (b, n) in zip(*np.nonzero(coin)):
                if status[b] < 2:
                    acts[b, n] = rng.choice(np.nonzero(av[b, n])[0])
            for b in range(B):
                if status[b] == 2:
                    continue
                bt["actions"][b, t, :, 0] = acts[b]
                bt["actions_onehot"][b, t, np.arange(NA), acts[b]] = 1.0
                if status[b] == 1:
                    status[b] = 2
                    continue
                rew, done, _ = envs[b].step(acts[b])
                env_steps += 1
                bt["reward"][b, t] = rew[0]
                bt["terminated"][b, t] = done
                observe(b, t + 1)
                if done:
                    status[b] = 1
            t += 1
        runs += 1
        for b in range(B):
            buffer.append({k: v[b] for k, v in bt.items()})
        del buffer[:-capacity]
        if len(buffer) >= batch_size:
            idx = rng.choice(len(buffer), batch_size, replace=False)
            smp = {k: torch.from_numpy(np.stack([buffer[i][k] for i in idx])) for k in buffer[0]}
            T = int(smp["filled"].sum(1).max())
            smp = {k: v[:, :T].clone() for k, v in smp.items()}
            groupA = torch.bernoulli(torch.rand(batch_size, 1, 1).repeat(1, 1, NE)).to(torch.uint8)
            learner.train(smp, groupA, runs * B)
            trains += 1
    elapsed = time.perf_counter() - t_start
    return {"value": env_steps / elapsed, "env_steps": env_steps, "seconds": elapsed, "runs": runs, "trains": trains,
            "cores": threads, "B": B}


def _env_worker(conn, env_kw):
    """EnvWorker.run (env_worker_process.py:27-71): a command loop over one env."""
    e = envref.RefEnv(**env_kw)
    while True:
        cmd, data = conn.recv()
        if cmd == "step":
            rew, done, info = e.step(data)
            conn.send((rew, done, info, e.state(), e.avail(), e.obs()))
        elif cmd == "reset":
            e.reset()
            conn.send((e.state(), e.avail(), e.obs()))
        elif cmd == "close":
            conn.close()
            return
        else:
            raise NotImplementedError(cmd)


def run_process_model(seconds=15.0, B=None, episode_limit=100, eps=0.05, threads=None, seed=0, batch_size=32,
                      capacity=512):
    """ParallelStepper.run in the reference's process model: B worker processes (one env each); per step the
    parent sends ("step", actions) to every running env, then receives every result (parallel_stepper.py:143-191),
    with the stepper bookkeeping of stepper_ref.run and one QLearner.train per run."""
    B = B or core_share()[0]
    threads = threads or B
    p = PLAN_MEDIUM_1H_4T
    U, N = 10, 5
    A, d_obs, S = 5 + U, 8 * U, 6 * U
    d_in = d_obs + A + N
    ctx = mp.get_context("fork")  # this process never touched a GPU; workers only run the C env
    conns, procs = [], []
    for b in range(B):
        a, w = ctx.Pipe()
        kw = dict(team=p["team"], role=p["role"], melee=p["melee"], scripted=p["scripted"],
                  episode_limit=episode_limit, seed=seed, env_index=b)
        pr = ctx.Process(target=_env_worker, args=(w, kw), daemon=True)
        pr.start()
        conns.append(a)
        procs.append(pr)
    torch.set_num_threads(threads)
    agent, mix = _init_params(d_in, 64, A, N, S, seed=seed)
    args = SimpleNamespace(n_agents=N, n_actions=A, mixer="qmix", mixing_embed_dim=32, hypernet_layers=2,
                           double_q=True, gamma=0.99, lr=5e-4, optim_alpha=0.99, optim_eps=1e-5, grad_norm_clip=10,
                           target_update_interval=200, obs_last_action=True, obs_agent_id=True)
    learner = LR.QLearnerRef(agent, mix, args)
    T1 = episode_limit + 1
    eye = torch.eye(N).unsqueeze(0).expand(B, -1, -1).reshape(B * N, N)
    buffer, rng = [], np.random.RandomState(seed)
    env_steps, runs, trains = 0, 0, 0
    t_start = time.perf_counter()
    try:
        while time.perf_counter() - t_start < seconds:
            batch = SR.new_batch(B, T1, N, A, d_obs, S)
            for c in conns:
                c.send(("reset", None))
            for i, c in enumerate(conns):
                batch["state"][i, 0], batch["avail_actions"][i, 0], batch["obs"][i, 0] = c.recv()
                batch["filled"][i, 0] = 1
            h = torch.zeros(B * N, 64)
            terminated = [False] * B
            running = list(range(B))
            t = 0
            while True:
                obs = torch.from_numpy(batch["obs"][:, t].reshape(B * N, d_obs))
                last = torch.from_numpy(batch["actions_onehot"][:, t - 1].reshape(B * N, A)) if t > 0 \
                    else torch.zeros(B * N, A)
                with torch.no_grad():  # forward on all B rows, selection on the running ones (:132-134)
                    q, h = LR.drqn_forward(learner.p, torch.cat([obs, last, eye], 1), h)
                ids = list(running)
                qv = q.view(B, N, A)[ids]
                av = torch.from_numpy(batch["avail_actions"][ids, t])
                acts = LR.greedy_select(qv, av).numpy()
                coin = rng.rand(*acts.shape) < eps
                for (k, n) in zip(*np.nonzero(coin)):
                    acts[k, n] = rng.choice(np.nonzero(av[k, n].numpy())[0])
                for k, i in enumerate(ids):
                    batch["actions"][i, t, :, 0] = acts[k]
                    batch["actions_onehot"][i, t, np.arange(N), acts[k]] = 1.0
                sent = [i for k, i in enumerate(ids) if not terminated[i]]
                for k, i in enumerate(ids):
                    if not terminated[i]:
                        conns[i].send(("step", acts[k]))
                running = [i for i in range(B) if not terminated[i]]
                if all(terminated):
                    break
                for i in sent:
                    rew, done, info, st, avl, ob = conns[i].recv()
                    env_steps += 1
                    terminated[i] = done
                    batch["reward"][i, t, 0] = rew[0]
                    batch["terminated"][i, t, 0] = done
                    batch["state"][i, t + 1], batch["avail_actions"][i, t + 1], batch["obs"][i, t + 1] = st, avl, ob
                    batch["filled"][i, t + 1] = 1
                t += 1
            runs += 1
            for b in range(B):
                buffer.append({k: v[b] for k, v in batch.items()})
            del buffer[:-capacity]
            if len(buffer) >= batch_size:
                idx = rng.choice(len(buffer), batch_size, replace=False)
                smp = {k: torch.from_numpy(np.stack([buffer[i][k] for i in idx])) for k in buffer[0]}
                T = int(smp["filled"].sum(1).max())
                smp = {k: v[:, :T].clone() for k, v in smp.items()}
                learner.train(smp, env_steps, runs * B)
                trains += 1
        elapsed = time.perf_counter() - t_start
    finally:
        for c in conns:
            try:
                c.send(("close", None))
            except OSError:
                pass
        for pr in procs:
            pr.join(timeout=5)
            if pr.is_alive():
                pr.terminate()
    return {"value": env_steps / elapsed, "env_steps": env_steps, "seconds": elapsed, "runs": runs, "trains": trains,
            "cores": threads, "B": B, "workers": B}


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or None


def _cgroup_cpus():
    """CPUs this process may use: the cgroup v2 quota (cpu.max) and the affinity mask, whichever is smaller."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def core_share():
    """Threads / env-worker processes of the CPU legs: this GPU's share of the host (host CPUs / 8 GPUs per node;
    VERDICT r4), capped by what the process may actually use (cgroup quota, affinity)."""
    share = max(1, (os.cpu_count() or 8) // 8)
    return min(share, _cgroup_cpus()), share


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", action="store_true")
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--episode-limit", type=int, default=100)
    ap.add_argument("--legs", default="vector,process")
    a = ap.parse_args(argv)
    threads, share = core_share()
    legs = []
    for leg in a.legs.split(","):
        if leg == "vector":
            r = run(seconds=a.seconds, B=64, episode_limit=a.episode_limit, threads=threads)
            what = "vectorised port: one process, oracle stepper + C env + PyTorch-CPU DRQN/QMIX learner"
        elif leg == "process":
            r = run_process_model(seconds=a.seconds, B=threads, episode_limit=a.episode_limit)
            what = (f"reference process model: {r['workers']} env-worker processes (one env each, pipe round trip "
                    f"per env per step) + PyTorch-CPU DRQN/QMIX learner in the parent")
        elif leg == "refil":
            r = run_refil(seconds=a.seconds, B=32, episode_limit=a.episode_limit, threads=threads)
            what = "C entity env + PyTorch-CPU EntityAttentionRNNAgent / REFILLearner (refil_ref)"
        else:
            raise SystemExit(f"unknown leg {leg}")
        legs.append({"leg": leg, "value": r["value"], "cores": r["cores"], "B": r["B"],
                     "sample": f"{r['runs']} runs x {r['B']} envs (+1 train each), {r['env_steps']} env steps in "
                               f"{r['seconds']:.1f}s; {what}"})
    out = {"legs": legs, "cpu_model": _cpu_model(), "host_cpus": os.cpu_count(), "per_gpu_core_share": share,
           "usable_cpus": _cgroup_cpus()}
    print(json.dumps(out) if a.json else out)


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    main()
