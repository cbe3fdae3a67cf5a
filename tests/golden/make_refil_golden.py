"""Generate REFIL golden vectors from the reference (config 5 layers + one REFILLearner.train step).

TEST INFRASTRUCTURE ONLY; runs in the build container with the reference mounted read-only at
/root/reference and records inputs/outputs of the reference's own modules as .npz data.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_refil_golden.py

refil_layers.npz
  attn.*      EntityAttentionLayer.forward + backward   src/marl/modules/layers/attention.py:24-79
              (nq = n_agents and nq = n_entities; rows with every entity masked -> NaN -> 0)
  agent.*     EntityAttentionRNNAgent.forward           src/marl/modules/agents/entity_rnn_agent.py:32-65
  imagine.*   ImagineEntityAttentionRNNAgent.forward    entity_rnn_agent.py:72-126 (the Bernoulli group draw
              is recorded: the build takes the groups as an input)
  mixer.*     FlexQMixer.forward (plain and with imagine groups; |w| and softmax mixing weights)
                                                        src/marl/modules/mixers/flex_qmix.py:36-117
refil_learner.npz
  REFILLearner.train (src/marl/learners/refil_learner.py:67-177), two consecutive calls. The reference's
  EntityMAC cannot serve ``forward(batch, t=None)`` (entity_controller.py:14-20 dereferences t.start; SURVEY
  §0.7); the fixture uses the intended semantics -- t=None means the whole episode, t = slice(0, T) -- with
  the reference's own EntityMAC._build_inputs and agent networks.
"""
import os
import sys
from types import SimpleNamespace

import numpy as np

REF_SRC = "/root/reference/src"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REF_SRC)
sys.dont_write_bytecode = True

import torch as th  # noqa: E402

th.set_num_threads(1)

# The reference targets torch 1.9 (run.sh:25), where masked_fill accepted uint8 masks (read as bool, with a
# deprecation warning); torch 2.x refuses them. Restore the 1.9 semantics for the generator only.
_masked_fill = th.Tensor.masked_fill


def _masked_fill_u8(self, mask, value):
    return _masked_fill(self, mask.bool() if mask.dtype == th.uint8 else mask, value)


th.Tensor.masked_fill = _masked_fill_u8

from marl.components.episode_batch import EpisodeBatch  # noqa: E402
from marl.components.transforms import OneHot  # noqa: E402
from marl.controllers.entity_controller import EntityMAC  # noqa: E402
from marl.learners.refil_learner import REFILLearner  # noqa: E402
from marl.modules.agents.entity_rnn_agent import EntityAttentionRNNAgent, ImagineEntityAttentionRNNAgent  # noqa: E402
from marl.modules.layers.attention import EntityAttentionLayer  # noqa: E402
from marl.modules.mixers.flex_qmix import FlexQMixer  # noqa: E402

NA, NE, ED, A = 8, 16, 8, 21  # agents, entities, entity features, actions


def refil_args(**kw):
    a = dict(n_agents=NA, n_entities=NE, n_actions=A, entity_shape=ED, entity_last_action=True,
             attn_embed_dim=64, attn_n_heads=4, rnn_hidden_dim=64, hypernet_embed=64, mixing_embed_dim=32,
             pooling_type=None, softmax_mixing_weights=False, mixer="flex_qmix", entity_scheme=True,
             agent="imagine_entity_attend_rnn", agent_output_type="q", action_selector="epsilon_greedy",
             epsilon_start=1.0, epsilon_finish=0.05, epsilon_anneal_time=50000, double_q=True, gamma=0.99,
             lr=5e-4, optim_alpha=0.99, optim_eps=1e-5, weight_decay=0, grad_norm_clip=10,
             target_update_interval=200, learner_log_interval=0, lmbda=0.5, train_gt_factors=False,
             train_rand_gt_factors=False, test_gt_factors=False, gt_mask_avail=False, device="cpu",
             obs_last_action=False, obs_agent_id=False, freeze_native=False)
    a.update(kw)
    return SimpleNamespace(**a)


def sd(prefix, module):
    return {f"{prefix}{k}": v.detach().numpy().copy() for k, v in module.state_dict().items()}


def entity_masks(rng, bs, n_active=None):
    """entity_mask [bs, NE] (1 = absent): n_active agents of 3..8 per team, rest padding; obs_mask from
    sight (random) over present entities."""
    em = np.ones((bs, NE), np.uint8)
    for b in range(bs):
        k = rng.randint(3, NA + 1) if n_active is None else n_active
        em[b, :k] = 0
        em[b, NA:NA + k] = 0
    om = (rng.rand(bs, NE, NE) < 0.3).astype(np.uint8)
    om |= em[:, None, :] | em[:, :, None]
    for b in range(bs):
        for i in range(NE):
            if not em[b, i]:
                om[b, i, i] = 0  # an active entity always sees itself
    return em, om


def attn_fixture(out, rng):
    args = refil_args()
    th.manual_seed(1)
    layer = EntityAttentionLayer(64, 64, 64, args)
    out.update(sd("attn.p.", layer))
    bs = 6
    x = th.tensor(rng.randn(bs, NE, 64).astype(np.float32), requires_grad=True)
    em, om = entity_masks(rng, bs)
    om[0, 2, :] = 1  # an active agent that sees nothing: softmax row of -inf -> NaN -> 0
    for tag, nq in (("na", NA), ("ne", NE)):
        post = th.tensor(em[:, :nq].astype(bool))
        pre = th.tensor(om.astype(bool))
        x.grad = None
        layer.zero_grad()
        y = layer(x, pre_mask=pre, post_mask=post)
        g = th.tensor(rng.randn(*y.shape).astype(np.float32))
        (y * g).sum().backward()
        out[f"attn.{tag}.y"] = y.detach().numpy()
        out[f"attn.{tag}.g"] = g.numpy()
        out[f"attn.{tag}.dx"] = x.grad.numpy().copy()
        for k, p in layer.named_parameters():
            out[f"attn.{tag}.d.{k}"] = p.grad.numpy().copy()
    out["attn.x"] = x.detach().numpy()
    out["attn.pre"] = om
    out["attn.em"] = em


def agent_fixture(out, rng):
    args = refil_args(agent="entity_attend_rnn")
    th.manual_seed(2)
    ag = EntityAttentionRNNAgent(ED + A, args)
    out.update(sd("agent.p.", ag))
    bs, ts = 4, 5
    ent = th.tensor(rng.randn(bs, ts, NE, ED + A).astype(np.float32))
    ems, oms = zip(*[entity_masks(rng, bs) for _ in range(ts)])
    em = np.stack(ems, 1)
    om = np.stack(oms, 1)
    h0 = th.tensor(rng.randn(bs, NA, 64).astype(np.float32))
    q, hs = ag((ent, th.tensor(om.astype(bool)), th.tensor(em.astype(bool))), h0)
    out.update({"agent.ent": ent.numpy(), "agent.om": om, "agent.em": em, "agent.h0": h0.numpy(),
                "agent.q": q.detach().numpy(), "agent.hs": hs.detach().numpy()})
    # imagination: record the Bernoulli draw (the build takes group membership as an input)
    args_i = refil_args()
    th.manual_seed(2)
    agi = ImagineEntityAttentionRNNAgent(ED + A, args_i)
    agi.load_state_dict(ag.state_dict())
    drawn = []
    orig = th.bernoulli

    def rec(p, *a, **k):
        r = orig(p, *a, **k)
        drawn.append(r.clone())
        return r

    th.bernoulli = rec
    th.manual_seed(3)
    qi, hi, (wm, im) = agi((ent, th.tensor(om.astype(bool)).to(th.uint8), th.tensor(em.astype(np.uint8))), h0,
                            imagine=True)
    th.bernoulli = orig
    out.update({"imagine.groupA": drawn[0].numpy().astype(np.uint8), "imagine.q": qi.detach().numpy(),
                "imagine.hs": hi.detach().numpy(), "imagine.Wmask": wm.numpy(), "imagine.Imask": im.numpy()})


def mixer_fixture(out, rng):
    for sm in (False, True):
        tag = "soft" if sm else "abs"
        args = refil_args(softmax_mixing_weights=sm)
        th.manual_seed(4)
        mx = FlexQMixer(args)
        out.update(sd(f"mixer.{tag}.p.", mx))
        bs, ts = 3, 4
        ent = th.tensor(rng.randn(bs, ts, NE, ED + A).astype(np.float32))
        em = np.stack([entity_masks(rng, bs)[0] for _ in range(ts)], 1)
        qs = th.tensor(rng.randn(bs, ts, NA).astype(np.float32))
        y = mx(qs, (ent, th.tensor(em.astype(np.uint8))))
        wm = (rng.rand(bs, ts, NE, NE) < 0.5).astype(np.uint8)
        im = 1 - wm
        qs2 = th.tensor(rng.randn(bs, ts, 2 * NA).astype(np.float32))
        y2 = mx(qs2, (ent, th.tensor(em.astype(np.uint8))), imagine_groups=(th.tensor(wm), th.tensor(im)))
        out.update({f"mixer.{tag}.ent": ent.numpy(), f"mixer.{tag}.em": em, f"mixer.{tag}.qs": qs.numpy(),
                    f"mixer.{tag}.y": y.detach().numpy(), f"mixer.{tag}.qs2": qs2.numpy(),
                    f"mixer.{tag}.wm": wm, f"mixer.{tag}.im": im, f"mixer.{tag}.y2": y2.detach().numpy()})


class _Log:
    def __init__(self):
        self.stats = {}
        self.console_logger = SimpleNamespace(info=lambda *a, **k: None)

    def log_stat(self, k, v, t):
        self.stats[k] = float(v)


class _IntendedEntityMAC(EntityMAC):
    """EntityMAC with the intended forward(batch, t=None, imagine=...) (REFIL's basic controller): t=None ->
    the whole episode; inputs from the reference's own EntityMAC._build_inputs."""

    def train(self):  # REFIL's controller forwards train()/eval() to the agent (refil_learner.py:82-85)
        self.agent.train()

    def eval(self):
        self.agent.eval()

    def forward(self, ep_batch, t=None, test_mode=False, imagine=False, **kw):
        if t is None:
            t = slice(0, ep_batch["avail_actions"].shape[1])
        inputs = self._build_inputs(ep_batch, t)
        if imagine:
            q, self.hidden_states, groups = self.agent(inputs, self.hidden_states, imagine=True)
            return q, groups
        q, self.hidden_states = self.agent(inputs, self.hidden_states)
        return q


def learner_fixture(rng):
    from marl.modules.agents import REGISTRY as agent_REGISTRY
    agent_REGISTRY["imagine_entity_attend_rnn"] = ImagineEntityAttentionRNNAgent
    args = refil_args()
    B, T = 4, 7
    scheme = {"entities": {"vshape": ED, "group": "entities"},
              "obs_mask": {"vshape": (NE,), "group": "entities", "dtype": th.uint8},
              "entity_mask": {"vshape": (NE,), "dtype": th.uint8},
              "actions": {"vshape": (1,), "group": "agents", "dtype": th.long},
              "avail_actions": {"vshape": (A,), "group": "agents", "dtype": th.int},
              "reward": {"vshape": (1,)}, "terminated": {"vshape": (1,), "dtype": th.uint8}}
    groups = {"agents": NA, "entities": NE}
    pre = {"actions": ("actions_onehot", [OneHot(out_dim=A)])}
    batch = EpisodeBatch(scheme, groups, B, T, preprocess=pre)
    lens = [6, 4, 6, 3]
    ent = rng.randn(B, T, NE, ED).astype(np.float32)
    ems, oms = zip(*[entity_masks(rng, B) for _ in range(T)])
    em, om = np.stack(ems, 1), np.stack(oms, 1)
    em[:] = em[:, :1]  # entity presence is fixed per episode
    om |= em[:, :, None, :] | em[:, :, :, None]
    avail = (rng.rand(B, T, NA, A) < 0.6).astype(np.int32)
    avail[..., 0] = 1
    acts = np.zeros((B, T, NA, 1), np.int64)
    for b in range(B):
        for t in range(T):
            for n in range(NA):
                acts[b, t, n, 0] = rng.choice(np.nonzero(avail[b, t, n])[0])
    rew = rng.randn(B, T, 1).astype(np.float32)
    for b, L in enumerate(lens):
        tt = th.from_numpy
        batch.update({"entities": tt(ent[b, :L + 1]), "obs_mask": tt(om[b, :L + 1]),
                      "entity_mask": tt(em[b, :L + 1]), "avail_actions": tt(avail[b, :L + 1])},
                     bs=b, ts=slice(0, L + 1))
        batch.update({"actions": tt(acts[b, :L + 1])}, bs=b, ts=slice(0, L + 1), mark_filled=False)
        term = np.zeros((L, 1), np.uint8)
        term[-1] = 1 if b != 2 else 0
        batch.update({"reward": tt(rew[b, :L]), "terminated": tt(term)}, bs=b, ts=slice(0, L), mark_filled=False)
    th.manual_seed(5)
    mac = _IntendedEntityMAC(batch.scheme, groups, args)
    learner = REFILLearner(mac, batch.scheme, _Log(), args)
    out = {f"b.{k}": v.numpy().copy() for k, v in batch.data.transition_data.items()}
    out.update(sd("p0.agent.", mac.agent))
    out.update(sd("p0.mixer.", learner.mixer))
    drawn = []
    orig = th.bernoulli

    def rec(p, *a, **k):
        r = orig(p, *a, **k)
        drawn.append(r.clone())
        return r

    th.bernoulli = rec
    for call in range(2):
        th.manual_seed(100 + call)
        learner.logger = _Log()
        learner.train(batch, t_env=1000 * (call + 1), episode_num=call)
        out[f"c{call}.groupA"] = drawn[-1].numpy().astype(np.uint8)
        for k, v in learner.logger.stats.items():
            out[f"c{call}.stat.{k}"] = np.array(v)
        out.update(sd(f"c{call}.agent.", mac.agent))
        out.update(sd(f"c{call}.mixer.", learner.mixer))
    th.bernoulli = orig
    np.savez_compressed(os.path.join(OUT, "refil_learner.npz"), **out)


def main():
    rng = np.random.RandomState(7)
    out = {}
    attn_fixture(out, rng)
    agent_fixture(out, rng)
    mixer_fixture(out, rng)
    np.savez_compressed(os.path.join(OUT, "refil_layers.npz"), **out)
    learner_fixture(rng)
    print("refil fixtures written to", OUT)


if __name__ == "__main__":
    main()
