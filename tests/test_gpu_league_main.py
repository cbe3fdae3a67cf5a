"""The league entry point (maleague/league/main.py; central_worker_main.py:28-111 + CentralWorker.run) end to end on
one MI355X: two ranks launched by torch.distributed.run, both players on cuda:0 over gloo (one GPU on this box),
each with its own composed team (force-unit HEALER / RANGED): pre-training against the mirrored scripted AI, then
league iterations whose every match plays the opponent's roster; the payoff counts every episode once."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("experiment,world,league_size", [("matchmaking", 2, 2), ("alphastar", 2, 1)])
def test_league_main_two_ranks_one_gpu(tmp_path, experiment, world, league_size):
    B, iters, per_match = 256, 3, 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}",
           os.path.join(ROOT, "ma-league_amd", "maleague", "league", "main.py"),
           "--backend=gloo", "--device=0", "--config=qmix", "--env-config=ma", "--league-config=matchmaking",
           f"--experiment={experiment}", f"--league_size={league_size}", "--team_size=5",
           f"--league-iterations={iters}", f"--match-iterations={per_match}", "--pretrain-iterations=1",
           "--runner=parallel", f"--batch_size_run={B}", "--env_args.episode_limit=30", "--buffer_size=512",
           "--league_checkpoint_min_steps=1", "--league_checkpoint_max_steps=1", f"--local_results_path={tmp_path}",
           "force-unit", "--role=HEALER", "--attack=RANGED"]
    env = dict(os.environ, OMP_NUM_THREADS="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env, cwd=str(tmp_path))
    assert p.returncode == 0, p.stderr[-3000:] + p.stdout[-2000:]
    s = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    players = s["players"]
    assert len(players) == world and all(pl["codes"].startswith("HR") for pl in players)
    if experiment == "matchmaking":
        assert players[0]["team"]["tid"] != players[1]["team"]["tid"]
    else:  # one team: a main player and its main exploiter
        assert [pl["role"] for pl in players] == ["main", "main_exploiter"]
        assert players[0]["team"] == players[1]["team"]
    assert s["league_iterations"] == iters
    for rank, matches in enumerate(s["matches"]):
        assert len(matches) == iters
        for m in matches:
            assert m["iterations"] == per_match
            parent = m["opponent"] if not m["historical"] else None
            if parent is not None:
                assert m["away_codes"] == players[parent]["codes"]
            assert m["away_codes"] in {pl["codes"] for pl in players}
    pay = s["payoff"]
    games = sum(pay[i][j][0] for i in range(len(pay)) for j in range(len(pay)))
    assert games == world * iters * per_match * B
    assert os.path.exists(os.path.join(s["log_dir"], "league_config.json"))
    assert "Stats for Team #" in p.stdout
