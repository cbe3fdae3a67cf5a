"""bench.py's league leg (the code path the driver's N-GPU runs time) over gloo on CPU, world size 2 and 4.

The learner is a stand-in (no GPU here): random battle outcomes, t_env / trained_steps counting. Everything
else is the product code bench.py runs: bench.run_league_leg -> timed_loop -> LeagueInstance.sync (payoff
all_reduce, parameter all_gather, barrier, matchmaking) every match_len iterations -> LeagueInstance.play."""
import os
import socket
import sys

import numpy as np
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _Agent(torch.nn.Module):
    def __init__(self, rank):
        super().__init__()
        self.w = torch.nn.Parameter(torch.full((6,), float(rank)))
        self.trained_steps = 0


class _MAC:
    def __init__(self, rank):
        self.agent = _Agent(rank)


class _Stepper:
    def __init__(self, B):
        self.batch_size = B
        self._info = torch.zeros(6 * B, dtype=torch.int32)
        self.t_env = 0
        self.agent_rows = torch.zeros(1, dtype=torch.int64)
        self.timing = None
        self.t_history = None
        self._run_id = 0


class _Experiment:
    def __init__(self, rank, B=16):
        self.home_mac, self.away_mac = _MAC(rank), _MAC(-1)
        self.stepper = _Stepper(B)
        self.rng = np.random.RandomState(rank)
        self.loaded = []

    def load_adversary_vector(self, vec):
        with torch.no_grad():
            self.away_mac.agent.w.copy_(vec)
        self.loaded.append(float(vec[0]))

    def _train_episode(self, episode):
        st = self.stepper
        B = st.batch_size
        st._info[B:3 * B] = torch.from_numpy(self.rng.randint(0, 2, 2 * B).astype(np.int32))
        st._info[3 * B:4 * B] = torch.from_numpy(self.rng.randint(0, 2, B).astype(np.int32))
        st.t_env += B * 7
        st.agent_rows += B * 5
        self.home_mac.agent.trained_steps += B * 10
        with torch.no_grad():
            self.home_mac.agent.w.add_(1.0)


def _worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "ma-league_amd"))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from types import SimpleNamespace
    from maleague.league import DistributedLeague, LeagueInstance
    args = SimpleNamespace(matchmaking="pfsp", league_checkpoint_min_steps=300, league_checkpoint_max_steps=600,
                           env_args={})
    lg = DistributedLeague(n_players=world, device="cpu", seed=0, max_historical=2)
    mode, roles = bench.league_setup(world, args)
    inst = LeagueInstance(args, None, lg, mode=mode, role=roles, seed=0, experiment=_Experiment(rank))
    ctx = bench.Ctx(dist, torch.device("cpu"))
    assert mode == "rolebased" and len(roles) == world
    r = bench.run_league_leg(ctx, inst, steps=12, warmup=3, match_len=2)
    out.put((rank, r, lg.payoff.tensor.numpy().tolist(), list(lg.historical_meta)))
    dist.destroy_process_group()


def _run(world):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _check(res, world):
    r0 = res[0][1]
    # 12 timed iterations of B = 16 envs x 7 steps on every rank; value = all ranks' steps / max time
    assert r0["env_steps"] == world * 12 * 16 * 7
    assert len(r0["per_rank"]) == world
    assert abs(r0["value"] - r0["env_steps"] / r0["elapsed"]) < 1e-6 * r0["value"]
    assert r0["league_iterations"] == 6  # match_len 2 -> league iterations at timed i = 0, 2, .., 10
    assert r0["collective_backend"] == "gloo" and r0["world_size"] == world
    for rank, r, pay, meta in res:
        assert r["elapsed"] == r0["elapsed"]  # max over ranks
        np.testing.assert_array_equal(np.array(pay), np.array(res[0][2]))
        assert meta == res[0][3]
    # every played episode is in the replicated payoff once the last exchange has run
    assert r0["payoff_games"] > 0
    # snapshots are taken and historical opponents played inside the timed league iterations
    assert r0["snapshots_taken"] > 0 and r0["historical_snapshots"] > 0
    assert any(r["historical_matches_timed_rank0"] > 0 for _, r, _, _ in res)


def test_bench_league_leg_gloo_world2():
    _check(_run(2), 2)


def test_bench_league_leg_gloo_world4_alphastar_eviction():
    res = _run(4)
    _check(res, 4)
    assert len(res[0][3]) <= 2  # capacity 2: snapshots evicted, never dropped
