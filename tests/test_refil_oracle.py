"""The REFIL oracle (oracle/refil_ref.py) against the reference's own golden vectors (CPU)."""
from types import SimpleNamespace

import numpy as np
import torch

import refil_ref as RR

TOL = dict(atol=1e-5, rtol=1e-4)


def refil_args(**kw):
    a = dict(n_agents=8, n_entities=16, n_actions=21, entity_shape=8, entity_last_action=True, attn_embed_dim=64,
             attn_n_heads=4, rnn_hidden_dim=64, hypernet_embed=64, mixing_embed_dim=32, pooling_type=None,
             softmax_mixing_weights=False, double_q=True, gamma=0.99, lr=5e-4, optim_alpha=0.99, optim_eps=1e-5,
             weight_decay=0, grad_norm_clip=10, target_update_interval=200, lmbda=0.5)
    a.update(kw)
    return SimpleNamespace(**a)


def params(d, prefix):
    return {k[len(prefix):]: torch.from_numpy(np.array(d[k])) for k in d.files if k.startswith(prefix)}


def test_attention_layer_forward_backward(golden):
    d = golden("refil_layers.npz")
    p = {k: v.requires_grad_(True) for k, v in params(d, "attn.p.").items()}
    em = torch.from_numpy(d["attn.em"]).bool()
    for tag, nq in (("na", 8), ("ne", 16)):
        x = torch.from_numpy(d["attn.x"]).requires_grad_(True)
        y = RR.attn_layer(p, x, torch.from_numpy(d["attn.pre"]).bool(), em[:, :nq], 4)
        np.testing.assert_allclose(y.detach().numpy(), d[f"attn.{tag}.y"], **TOL)
        for v in p.values():
            v.grad = None
        (y * torch.from_numpy(d[f"attn.{tag}.g"])).sum().backward()
        np.testing.assert_allclose(x.grad.numpy(), d[f"attn.{tag}.dx"], **TOL)
        for k, v in p.items():
            if f"attn.{tag}.d.{k}" in d.files:  # (scale_factor is a buffer)
                np.testing.assert_allclose(v.grad.numpy(), d[f"attn.{tag}.d.{k}"], **TOL)


def test_entity_agent_and_imagination(golden):
    d = golden("refil_layers.npz")
    p = params(d, "agent.p.")
    a = refil_args()
    ent, om, em = (torch.from_numpy(d[k]) for k in ("agent.ent", "agent.om", "agent.em"))
    h0 = torch.from_numpy(d["agent.h0"])
    q, hs = RR.entity_agent(p, ent, om, em, h0, a)
    np.testing.assert_allclose(q.detach().numpy(), d["agent.q"], **TOL)
    np.testing.assert_allclose(hs.detach().numpy(), d["agent.hs"], **TOL)
    within, interact, Wn, In = RR.imagine_masks(torch.from_numpy(d["imagine.groupA"]), em.to(torch.uint8),
                                                om.to(torch.uint8))
    ts = ent.shape[1]
    np.testing.assert_array_equal(Wn.repeat(1, ts, 1, 1).numpy(), d["imagine.Wmask"])
    np.testing.assert_array_equal(In.repeat(1, ts, 1, 1).numpy(), d["imagine.Imask"])
    qi, _ = RR.entity_agent(p, ent.repeat(3, 1, 1, 1), torch.cat([om.to(torch.uint8), within, interact], 0),
                            em.repeat(3, 1, 1), h0.repeat(3, 1, 1), a)
    np.testing.assert_allclose(qi.detach().numpy(), d["imagine.q"], **TOL)


def test_flex_qmixer(golden):
    d = golden("refil_layers.npz")
    for tag in ("abs", "soft"):
        a = refil_args(softmax_mixing_weights=tag == "soft")
        p = params(d, f"mixer.{tag}.p.")
        ent, em = torch.from_numpy(d[f"mixer.{tag}.ent"]), torch.from_numpy(d[f"mixer.{tag}.em"])
        y = RR.flex_qmix(p, torch.from_numpy(d[f"mixer.{tag}.qs"]), ent, em, a)
        np.testing.assert_allclose(y.detach().numpy(), d[f"mixer.{tag}.y"], **TOL)
        y2 = RR.flex_qmix(p, torch.from_numpy(d[f"mixer.{tag}.qs2"]), ent, em, a,
                          imagine_groups=(torch.from_numpy(d[f"mixer.{tag}.wm"]), torch.from_numpy(d[f"mixer.{tag}.im"])))
        np.testing.assert_allclose(y2.detach().numpy(), d[f"mixer.{tag}.y2"], **TOL)


def test_refil_learner_two_calls(golden):
    d = golden("refil_learner.npz")
    a = refil_args()
    batch = {k[2:]: torch.from_numpy(np.array(d[k])) for k in d.files if k.startswith("b.")}
    L = RR.REFILLearnerRef(params(d, "p0.agent."), params(d, "p0.mixer."), a)
    for call in range(2):
        st = L.train(batch, torch.from_numpy(d[f"c{call}.groupA"]), episode_num=call)
        for k, v in st.items():
            np.testing.assert_allclose(v, float(d[f"c{call}.stat.{k}"]), rtol=1e-4, atol=1e-6, err_msg=k)
        for k, v in L.agent.items():
            np.testing.assert_allclose(v.detach().numpy(), d[f"c{call}.agent.{k}"], atol=2e-5, rtol=0, err_msg=k)
        for k, v in L.mixer.items():
            np.testing.assert_allclose(v.detach().numpy(), d[f"c{call}.mixer.{k}"], atol=2e-5, rtol=0, err_msg=k)
