"""League host logic: payoff/PFSP against golden vectors (reference PayoffWrapper + PFSPSampling) and the
one-learner-per-rank exchange with world_size 2 over gloo on CPU."""
import os
import socket

import numpy as np
import torch
import torch.multiprocessing as mp


def test_pfsp_against_golden(golden):
    from maleague.league import PayoffWrapper, PFSPSampling
    d = golden("pfsp.npz")
    payoff = torch.from_numpy(np.array(d["payoff"]))
    wrap = PayoffWrapper(payoff.clone())
    samp = PFSPSampling()
    for i in range(payoff.shape[0]):
        np.testing.assert_allclose(wrap.win_rates(i).numpy(), d[f"win_rates{i}"], rtol=1e-6)
        np.testing.assert_allclose(wrap.win_rates(i, [0, 2, 4]).numpy(), d[f"win_rates_idx{i}"], rtol=1e-6)
        for w in ["linear", "squared", "variance", "linear_capped"]:
            np.testing.assert_allclose(samp.probabilities(d[f"win_rates{i}"], w), d[f"p{i}.{w}"], rtol=1e-6)


def test_record_result_and_reference_compat():
    from maleague.league import PayoffEntry, PayoffWrapper, episode_result
    p = PayoffWrapper(torch.zeros(3, 3, 5))
    p.record_result(0, 1, PayoffEntry.WIN)
    p.record_result(0, 1, PayoffEntry.DRAW)
    assert p.win_rates(0)[1].item() == 0.75 and p.win_rates(0)[2].item() == 0.5
    q = PayoffWrapper(torch.zeros(3, 3, 5), reference_compat=True)
    q.record_result(0, 1, PayoffEntry.WIN)
    assert q.win_rates(0)[1].item() == 0.5  # the reference's GAMES is never incremented
    assert episode_result({"battle_won": [True, False], "draw": False}) == PayoffEntry.WIN
    assert episode_result({"battle_won": [False, True], "draw": False}) == PayoffEntry.LOSS
    assert episode_result({"battle_won": [True, True], "draw": False}) == PayoffEntry.DRAW
    assert episode_result({"battle_won": [False, False], "draw": True}) == PayoffEntry.DRAW


def _worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from maleague.league import DistributedLeague, PayoffEntry
    lg = DistributedLeague(n_players=world, device="cpu", seed=0)
    params = torch.full((7,), float(rank + 1))
    allp = lg.share_params(params)
    lg.record(lg.player(), (lg.player() + 1) % world, PayoffEntry.WIN if rank == 0 else PayoffEntry.LOSS, n=2)
    lg.record_match(lg.player(), (lg.player() + 1) % world)
    pay = lg.sync_payoff().clone()
    opp = lg.pfsp_opponent()
    lg.barrier()
    out.put((rank, [p.tolist() for p in allp], pay.numpy().tolist(), opp))
    dist.destroy_process_group()


def test_distributed_league_gloo_world2():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in procs])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, p0, pay0, _), (r1, p1, pay1, _) = res
    assert p0 == p1 == [[1.0] * 7, [2.0] * 7]
    assert pay0 == pay1  # replicated payoff identical on every rank
    pay = np.array(pay0)
    assert pay[0, 1, 0] == 2 and pay[0, 1, 1] == 2 and pay[1, 0, 0] == 2 and pay[1, 0, 2] == 2
    assert pay[0, 1, 4] == 1 and pay[1, 0, 4] == 1
