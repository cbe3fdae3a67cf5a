"""CPU restatement (PyTorch fp32, autograd) of the reference's REFIL path (config 5).

TEST INFRASTRUCTURE ONLY: imported by tests/ as the checker; never by the product. Pinned against
tests/golden/refil_*.npz, generated from the reference itself by tests/golden/make_refil_golden.py.
Parameters are plain dicts keyed like the reference modules' state_dicts. Paths relative to
/root/reference/src.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def attn_layer(p, x, pre_mask, post_mask, n_heads, prefix=""):
    """EntityAttentionLayer.forward (marl/modules/layers/attention.py:24-79). x [bs, ne, in]; pre_mask
    [bs, >=nq, >=ne] bool (True = masked); post_mask [bs, nq] bool."""
    bs, ne, _ = x.shape
    nq = post_mask.shape[1]
    pre = pre_mask[:, :nq, :ne].bool()
    q, k, v = F.linear(x, p[prefix + "in_trans.weight"]).chunk(3, dim=2)
    E = q.shape[-1]
    hd = E // n_heads
    q = q[:, :nq].reshape(bs, nq, n_heads, hd).transpose(1, 2)
    k = k.reshape(bs, ne, n_heads, hd).transpose(1, 2)
    v = v.reshape(bs, ne, n_heads, hd).transpose(1, 2)
    logits = torch.matmul(q, k.transpose(2, 3)) / torch.tensor(float(hd)).sqrt()
    w = F.softmax(logits.masked_fill(pre.unsqueeze(1), -float("inf")), dim=3)
    w = w.masked_fill(w != w, 0)  # rows with every entity masked -> NaN -> 0 (:59)
    o = torch.matmul(w, v).transpose(1, 2).reshape(bs, nq, E)
    y = F.linear(o, p[prefix + "out_trans.weight"], p[prefix + "out_trans.bias"])
    return y.masked_fill(post_mask.bool().unsqueeze(2), 0)


def entity_to_attn_mask(m):
    """1 - (1-m_i)(1-m_j): pair masked if either entity is absent (entity_rnn_agent.py:85-91)."""
    a = 1 - m.float()
    return (1 - a.unsqueeze(-1) * a.unsqueeze(-2)).to(torch.uint8)


def hypernet(p, prefix, entities, entity_mask, n_agents, n_heads, mode, attn_mask=None):
    """AttentionHyperNet.forward (marl/modules/mixers/flex_qmix.py:36-53)."""
    x1 = F.relu(F.linear(entities, p[prefix + "fc1.weight"], p[prefix + "fc1.bias"]))
    agent_mask = entity_mask[:, :n_agents].bool()
    if attn_mask is None:
        attn_mask = 1 - torch.bmm((1 - agent_mask.float()).unsqueeze(2), (1 - entity_mask.float()).unsqueeze(1))
    x2 = attn_layer(p, x1, attn_mask.bool(), agent_mask, n_heads, prefix + "attn.")
    x3 = F.linear(x2, p[prefix + "fc2.weight"], p[prefix + "fc2.bias"]).masked_fill(agent_mask.unsqueeze(2), 0)
    if mode == "vector":
        return x3.mean(dim=1)
    if mode == "alt_vector":
        return x3.mean(dim=2)
    if mode == "scalar":
        return x3.mean(dim=(1, 2))
    return x3


def flex_qmix(p, agent_qs, entities, entity_mask, args, imagine_groups=None, prefix=""):
    """FlexQMixer.forward (flex_qmix.py:73-117)."""
    bs, max_t, ne, ed = entities.shape
    na, E, nh = args.n_agents, args.mixing_embed_dim, args.attn_n_heads
    entities = entities.reshape(bs * max_t, ne, ed)
    entity_mask = entity_mask.reshape(bs * max_t, ne)
    hn = lambda name, mode, am=None: hypernet(p, prefix + name + ".", entities, entity_mask, na, nh, mode, am)  # noqa
    if imagine_groups is not None:
        agent_qs = agent_qs.reshape(-1, 1, na * 2)
        Wm, Im = imagine_groups
        w1 = torch.cat([hn("hyper_w_1", "matrix", Wm.reshape(bs * max_t, ne, ne)),
                        hn("hyper_w_1", "matrix", Im.reshape(bs * max_t, ne, ne))], dim=1)
    else:
        agent_qs = agent_qs.reshape(-1, 1, na)
        w1 = hn("hyper_w_1", "matrix")
    b1 = hn("hyper_b_1", "vector").view(-1, 1, E)
    w1 = w1.view(bs * max_t, -1, E)
    w1 = F.softmax(w1, dim=-1) if args.softmax_mixing_weights else torch.abs(w1)
    hidden = F.elu(torch.bmm(agent_qs, w1) + b1)
    wf = hn("hyper_w_final", "vector")
    wf = (F.softmax(wf, dim=-1) if args.softmax_mixing_weights else torch.abs(wf)).view(-1, E, 1)
    v = hn("V", "scalar").view(-1, 1, 1)
    return (torch.bmm(hidden, wf) + v).view(bs, -1, 1)


def gru_cell(p, x, h, prefix="rnn."):
    """torch.nn.GRUCell (gate order r, z, n)."""
    H = h.shape[-1]
    gi = F.linear(x, p[prefix + "weight_ih"], p[prefix + "bias_ih"])
    gh = F.linear(h, p[prefix + "weight_hh"], p[prefix + "bias_hh"])
    r = torch.sigmoid(gi[:, :H] + gh[:, :H])
    z = torch.sigmoid(gi[:, H:2 * H] + gh[:, H:2 * H])
    n = torch.tanh(gi[:, 2 * H:] + r * gh[:, 2 * H:])
    return n + z * (h - n)


def entity_agent(p, entities, obs_mask, entity_mask, h0, args):
    """EntityAttentionRNNAgent.forward (marl/modules/agents/entity_rnn_agent.py:32-65) -> q [bs,ts,na,A], hs."""
    bs, ts, ne, ed = entities.shape
    na, H = args.n_agents, args.rnn_hidden_dim
    ent = entities.reshape(bs * ts, ne, ed)
    om = obs_mask.reshape(bs * ts, ne, ne).bool()
    em = entity_mask.reshape(bs * ts, ne).bool()
    agent_mask = em[:, :na]
    x1 = F.relu(F.linear(ent, p["fc1.weight"], p["fc1.bias"]))
    x2 = attn_layer(p, x1, om, agent_mask, args.attn_n_heads, "attn.")
    x3 = F.relu(F.linear(x2, p["fc2.weight"], p["fc2.bias"])).reshape(bs, ts, na, -1)
    h = h0.reshape(-1, H)
    hs = []
    for t in range(ts):
        h = gru_cell(p, x3[:, t].reshape(-1, H), h)
        hs.append(h.reshape(bs, na, H))
    hs = torch.stack(hs, dim=1)
    q = F.linear(hs, p["fc3.weight"], p["fc3.bias"]).reshape(bs, ts, na, -1)
    return q.masked_fill(agent_mask.reshape(bs, ts, na, 1), 0), hs


def imagine_masks(groupA_raw, entity_mask, obs_mask):
    """ImagineEntityAttentionRNNAgent.forward mask algebra (entity_rnn_agent.py:93-118) for a given Bernoulli
    draw groupA_raw [bs, 1, ne] (uint8): returns (obs masks of the within / interact copies, W and I mixer
    masks without observability)."""
    lor = lambda a, b: ((a.int() + b.int()) > 0).to(torch.uint8)  # noqa: E731
    lnot = lambda a: (1 - a.int()).to(torch.uint8)  # noqa: E731
    em0 = entity_mask[:, [0]].to(torch.uint8)
    gA = lor(groupA_raw, em0)
    gB = lor(lnot(groupA_raw), em0)
    interact = lor(lnot(entity_to_attn_mask(gA)), lnot(entity_to_attn_mask(gB)))
    within = lnot(interact)
    active = entity_to_attn_mask(em0)
    W_noobs, I_noobs = lor(within, active), lor(interact, active)
    return lor(within, obs_mask), lor(interact, obs_mask), W_noobs, I_noobs


def build_entity_inputs(batch, n_agents, n_actions, T=None):
    """EntityMAC._build_inputs for t = slice(0, T) (entity_controller.py:11-30, intended t=None semantics)."""
    ent = batch["entities"]
    bs, T_all = ent.shape[:2]
    T = T_all if T is None else T
    ent = ent[:, :T]
    acs = torch.zeros(bs, T, ent.shape[2], n_actions, dtype=ent.dtype)
    acs[:, 1:, :n_agents] = batch["actions_onehot"][:, :T - 1]
    return torch.cat([ent, acs], dim=3), batch["obs_mask"][:, :T], batch["entity_mask"][:, :T]


def mac_forward(p, batch, args, groupA=None):
    """The whole-episode EntityMAC forward; with groupA, the imagined within / interact copies as well."""
    ent, om, em = build_entity_inputs(batch, args.n_agents, args.n_actions)
    bs = ent.shape[0]
    h0 = torch.zeros(bs, args.n_agents, args.rnn_hidden_dim)
    if groupA is None:
        return entity_agent(p, ent, om, em, h0, args)[0], None
    within, interact, Wn, In = imagine_masks(groupA, em, om)
    T = ent.shape[1]
    q, _ = entity_agent(p, ent.repeat(3, 1, 1, 1), torch.cat([om.to(torch.uint8), within, interact], dim=0),
                        em.repeat(3, 1, 1), h0.repeat(3, 1, 1), args)
    return q, (Wn.repeat(1, T, 1, 1), In.repeat(1, T, 1, 1))


class REFILLearnerRef:
    """REFILLearner.train (marl/learners/refil_learner.py:67-177) with RMSprop (learner ctor :34-35)."""

    def __init__(self, agent_p, mixer_p, args):
        self.args = args
        keep = lambda k: not k.endswith("scale_factor")  # noqa: E731  (a buffer, not a parameter)
        self.agent = {k: torch.as_tensor(v).clone().requires_grad_(True) for k, v in agent_p.items() if keep(k)}
        self.mixer = {k: torch.as_tensor(v).clone().requires_grad_(True) for k, v in mixer_p.items() if keep(k)}
        self.t_agent = {k: v.detach().clone() for k, v in self.agent.items()}
        self.t_mixer = {k: v.detach().clone() for k, v in self.mixer.items()}
        self.params = list(self.agent.values()) + list(self.mixer.values())
        self.opt = torch.optim.RMSprop(self.params, lr=args.lr, alpha=args.optim_alpha, eps=args.optim_eps,
                                       weight_decay=getattr(args, "weight_decay", 0))
        self.last_target_update_episode = 0

    def mixer_ins(self, batch):
        ent = batch["entities"]
        bs, T, ne, _ = ent.shape
        la = torch.zeros(bs, T, ne, self.args.n_actions)
        la[:, 1:, :self.args.n_agents] = batch["actions_onehot"][:, :-1]
        ent = torch.cat([ent, la], dim=3)
        em = batch["entity_mask"]
        return (ent[:, :-1], em[:, :-1]), (ent[:, 1:], em[:, 1:])

    def train(self, batch, groupA, episode_num):
        a = self.args
        rewards = batch["reward"][:, :-1]
        actions = batch["actions"][:, :-1]
        terminated = batch["terminated"][:, :-1].float()
        mask = batch["filled"][:, :-1].float()
        mask[:, 1:] = mask[:, 1:] * (1 - terminated[:, :-1])
        avail = batch["avail_actions"]
        all_q, groups = mac_forward(self.agent, batch, a, groupA=groupA)
        all_chosen = torch.gather(all_q[:, :-1], dim=3, index=actions.repeat(3, 1, 1, 1)).squeeze(3)
        mac_out = all_q.chunk(3, dim=0)[0]
        caq, caqW, caqI = all_chosen.chunk(3, dim=0)
        caq_imagine = torch.cat([caqW, caqI], dim=2)
        with torch.no_grad():
            tq, _ = mac_forward(self.t_agent, batch, a)
        tq = tq[:, 1:].clone()
        tq[avail[:, 1:] == 0] = -9999999
        if a.double_q:
            mo = mac_out.clone().detach()
            mo[avail == 0] = -9999999
            cur = mo[:, 1:].max(dim=3, keepdim=True)[1]
            tmax = torch.gather(tq, 3, cur).squeeze(3)
        else:
            tmax = tq.max(dim=3)[0]
        mix_ins, targ_ins = self.mixer_ins(batch)
        chosen = flex_qmix(self.mixer, caq, *mix_ins, a)
        groups = [g[:, :-1] for g in groups]
        caq_imagine = flex_qmix(self.mixer, caq_imagine, *mix_ins, a, imagine_groups=groups)
        with torch.no_grad():
            tmax = flex_qmix(self.t_mixer, tmax, *targ_ins, a)
        targets = rewards + a.gamma * (1 - terminated) * tmax
        td = chosen - targets.detach()
        mask = mask.expand_as(td)
        mtd = td * mask
        loss = (mtd ** 2).sum() / mask.sum()
        im_td = (caq_imagine - targets.detach()) * mask
        im_loss = (im_td ** 2).sum() / mask.sum()
        loss = (1 - a.lmbda) * loss + a.lmbda * im_loss
        self.opt.zero_grad()
        loss.backward()
        gn = torch.nn.utils.clip_grad_norm_(self.params, a.grad_norm_clip)
        self.opt.step()
        if (episode_num - self.last_target_update_episode) / a.target_update_interval >= 1.0:
            self.t_agent = {k: v.detach().clone() for k, v in self.agent.items()}
            self.t_mixer = {k: v.detach().clone() for k, v in self.mixer.items()}
            self.last_target_update_episode = episode_num
        me = mask.sum().item()
        return {"loss": loss.item(), "im_loss": im_loss.item(), "grad_norm": float(gn),
                "td_error_abs": mtd.abs().sum().item() / me,
                "q_taken_mean": (chosen * mask).sum().item() / (me * a.n_agents),
                "target_mean": (targets * mask).sum().item() / (me * a.n_agents)}


def softmax_scale(hd):  # documentation helper: the reference divides logits by sqrt(head_dim)
    return math.sqrt(hd)
