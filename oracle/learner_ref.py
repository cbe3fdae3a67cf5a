"""CPU restatement (PyTorch fp32, autograd) of the reference's QMIX learner path.

TEST INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as
the checker / CPU baseline; never by the product. Pinned against golden vectors generated from the
reference itself (tests/golden/make_golden.py -> tests/golden/*.npz).

Each function cites the reference lines it restates (paths relative to /root/reference/src).
"""
from __future__ import annotations

import copy

import numpy as np
import torch
import torch.nn.functional as F

AGENT_KEYS = ["fc1.weight", "fc1.bias", "gru.weight_ih", "gru.weight_hh", "gru.bias_ih", "gru.bias_hh",
              "fc2.weight", "fc2.bias"]


def drqn_forward(p, inputs, h):
    """marl/modules/agents/drqn_agent.py:29-35 (fc1 -> relu -> GRUCell -> fc2)."""
    x = F.relu(F.linear(inputs, p["fc1.weight"], p["fc1.bias"]))
    H = p["gru.weight_hh"].shape[1]
    h = h.reshape(-1, H)
    gi = F.linear(x, p["gru.weight_ih"], p["gru.bias_ih"])
    gh = F.linear(h, p["gru.weight_hh"], p["gru.bias_hh"])
    r = torch.sigmoid(gi[:, :H] + gh[:, :H])
    z = torch.sigmoid(gi[:, H:2 * H] + gh[:, H:2 * H])
    n = torch.tanh(gi[:, 2 * H:] + r * gh[:, 2 * H:])
    h_new = n + z * (h - n)  # torch GRUCell: (hx - newgate) * inputgate + newgate
    return F.linear(h_new, p["fc2.weight"], p["fc2.bias"]), h_new


def build_inputs(batch, t, n_agents, last_action=True, agent_id=True):
    """marl/controllers/basic_controller.py:80-92."""
    obs = batch["obs"][:, t]
    B = obs.shape[0]
    parts = [obs]
    if last_action:
        oh = batch["actions_onehot"]
        parts.append(torch.zeros_like(oh[:, t]) if t == 0 else oh[:, t - 1])
    if agent_id:
        parts.append(torch.eye(n_agents).unsqueeze(0).expand(B, -1, -1))
    return torch.cat([x.reshape(B * n_agents, -1) for x in parts], dim=1)


def mac_unroll(p, batch, n_agents, T=None, h0=None, last_action=True, agent_id=True):
    """BasicMAC.forward over t = 0..T-1 (basic_controller.py:38-54) -> [B, T, N, A]."""
    B = batch["obs"].shape[0]
    T = batch["obs"].shape[1] if T is None else T
    H = p["gru.weight_hh"].shape[1]
    h = torch.zeros(B * n_agents, H) if h0 is None else h0
    outs = []
    for t in range(T):
        q, h = drqn_forward(p, build_inputs(batch, t, n_agents, last_action, agent_id), h)
        outs.append(q.view(B, n_agents, -1))
    return torch.stack(outs, dim=1), h


def greedy_select(q, avail):
    """EpsilonGreedyActionSelector.select with test_mode=True (action_selectors.py:44-62, epsilon 0)."""
    m = q.clone()
    m[avail == 0] = -float("inf")
    return m.max(dim=-1)[1]


def eps_select(q, avail, eps, keys, episodes, t):
    """Epsilon-greedy with the build's counter-based stream in place of torch RNG:
    per agent row, u_eps = u01(rng(key, ctr(episode, t, 2, n))) < eps -> k-th available action with
    k from rng(key, ctr(episode, t, 3, n)). Rows are [env, agent]."""
    import envref  # oracle/envref.py
    greedy = greedy_select(q, avail).numpy()
    B, N = greedy.shape
    out = greedy.copy()
    is_greedy = np.ones_like(out)
    for e in range(B):
        for n in range(N):
            r1 = envref.rng(keys[e], envref.ctr(episodes[e], t, 2, n))
            if envref.u01(r1) < np.float32(eps):
                r2 = envref.rng(keys[e], envref.ctr(episodes[e], t, 3, n))
                out[e, n] = envref.random_available(avail[e, n].tolist(), r2)
                is_greedy[e, n] = 0
    return out, is_greedy


def qmix_forward(mp, agent_qs, states, n_agents, embed_dim, hypernet_layers=2):
    """marl/modules/mixers/qmix.py:41-59."""
    bs = agent_qs.size(0)
    S = states.shape[-1]
    s = states.reshape(-1, S)
    qs = agent_qs.reshape(-1, 1, n_agents)

    def mlp(prefix, x):
        if hypernet_layers == 2:
            return F.linear(F.relu(F.linear(x, mp[f"{prefix}.0.weight"], mp[f"{prefix}.0.bias"])),
                            mp[f"{prefix}.2.weight"], mp[f"{prefix}.2.bias"])
        return F.linear(x, mp[f"{prefix}.weight"], mp[f"{prefix}.bias"])

    w1 = torch.abs(mlp("hyper_w_1", s)).view(-1, n_agents, embed_dim)
    b1 = F.linear(s, mp["hyper_b_1.weight"], mp["hyper_b_1.bias"]).view(-1, 1, embed_dim)
    hidden = F.elu(torch.bmm(qs, w1) + b1)
    wf = torch.abs(mlp("hyper_w_final", s)).view(-1, embed_dim, 1)
    v = F.linear(F.relu(F.linear(s, mp["V.0.weight"], mp["V.0.bias"])), mp["V.2.weight"], mp["V.2.bias"]).view(-1, 1, 1)
    return (torch.bmm(hidden, wf) + v).view(bs, -1, 1)


class QLearnerRef:
    """QLearner.train + update_targets (marl/learners/q_learner.py:34-131), RMSprop (learner.py:25-31),
    clip_grad_norm_ (q_learner.py:104)."""

    def __init__(self, agent_params: dict, mixer_params: dict | None, args):
        self.args = args
        self.p = {k: torch.tensor(np.asarray(v), dtype=torch.float32).requires_grad_(True) for k, v in agent_params.items()}
        self.mixer = args.mixer
        self.mp = None
        if mixer_params is not None and args.mixer == "qmix":
            self.mp = {k: torch.tensor(np.asarray(v), dtype=torch.float32).requires_grad_(True)
                       for k, v in mixer_params.items()}
        self.tp = {k: v.detach().clone() for k, v in self.p.items()}
        self.tmp = None if self.mp is None else {k: v.detach().clone() for k, v in self.mp.items()}
        params = list(self.p.values()) + (list(self.mp.values()) if self.mp is not None else [])
        self.params = params
        self.opt = torch.optim.RMSprop(params, lr=args.lr, alpha=args.optim_alpha, eps=args.optim_eps)
        self.last_target_update_episode = 0
        self.trained_steps = 0

    def _mix(self, mp, qs, states):
        if self.mixer == "qmix":
            return qmix_forward(mp, qs, states, self.args.n_agents, self.args.mixing_embed_dim,
                                getattr(self.args, "hypernet_layers", 1))
        if self.mixer == "vdn":
            return torch.sum(qs, dim=2, keepdim=True)
        return qs

    def train(self, batch: dict, t_env: int, episode_num: int) -> dict:
        a = self.args
        N = a.n_agents
        rewards = batch["reward"][:, :-1]
        actions = batch["actions"][:, :-1]
        terminated = batch["terminated"][:, :-1].float()
        mask = batch["filled"][:, :-1].float()
        mask[:, 1:] = mask[:, 1:] * (1 - terminated[:, :-1])
        avail = batch["avail_actions"]
        T = batch["obs"].shape[1]
        mac_out, _ = mac_unroll(self.p, batch, N, T, last_action=a.obs_last_action, agent_id=a.obs_agent_id)
        chosen = torch.gather(mac_out[:, :-1], dim=3, index=actions).squeeze(3)
        with torch.no_grad():
            tmac, _ = mac_unroll(self.tp, batch, N, T, last_action=a.obs_last_action, agent_id=a.obs_agent_id)
        tmac = tmac[:, 1:].clone()
        tmac[avail[:, 1:] == 0] = -9999999
        if a.double_q:
            md = mac_out.clone().detach()
            md[avail == 0] = -9999999
            cur_max = md[:, 1:].max(dim=3, keepdim=True)[1]
            target_max = torch.gather(tmac, 3, cur_max).squeeze(3)
        else:
            target_max = tmac.max(dim=3)[0]
        if self.mixer in ("qmix", "vdn"):
            chosen = self._mix(self.mp, chosen, batch["state"][:, :-1])
            with torch.no_grad():
                target_max = self._mix(self.tmp, target_max, batch["state"][:, 1:])
        targets = rewards + a.gamma * (1 - terminated) * target_max
        td = chosen - targets.detach()
        mask = mask.expand_as(td)
        mtd = td * mask
        loss = (mtd ** 2).sum() / mask.sum()
        self.opt.zero_grad()
        loss.backward()
        grad_norm = torch.nn.utils.clip_grad_norm_(self.params, a.grad_norm_clip)
        self.opt.step()
        if (episode_num - self.last_target_update_episode) / a.target_update_interval >= 1.0:
            self.update_targets()
            self.last_target_update_episode = episode_num
        self.trained_steps += int(torch.count_nonzero(mask))
        me = mask.sum().item()
        return {"loss": loss.item(), "grad_norm": float(grad_norm), "td_error_abs": mtd.abs().sum().item() / me,
                "q_taken_mean": (chosen * mask).sum().item() / (me * N),
                "target_mean": (targets * mask).sum().item() / (me * N)}

    def update_targets(self):
        self.tp = {k: v.detach().clone() for k, v in self.p.items()}
        if self.mp is not None:
            self.tmp = {k: v.detach().clone() for k, v in self.mp.items()}

    def agent_state(self):
        return {k: v.detach().clone() for k, v in self.p.items()}

    def mixer_state(self):
        return None if self.mp is None else {k: v.detach().clone() for k, v in self.mp.items()}


def batch_from_npz(d, prefix="b."):
    """Golden-fixture batch dict (numpy) -> torch tensors with the scheme dtypes."""
    out = {}
    for k in d.files:
        if k.startswith(prefix):
            out[k[len(prefix):]] = torch.from_numpy(np.array(d[k]))
    return out


def clone_args(args, **kw):
    a = copy.copy(args)
    for k, v in kw.items():
        setattr(a, k, v)
    return a
