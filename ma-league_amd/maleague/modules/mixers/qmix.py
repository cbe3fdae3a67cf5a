"""QMIX hypernetwork mixer (API + state_dict keys of src/marl/modules/mixers/qmix.py:8-59).

Training runs the mixer forward/backward inside the fused learner kernels (learner.hip mix_td_kernel);
QMixer.forward here is the stand-alone inference path (mlg_qmix_forward).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from ... import _native


class QMixer(nn.Module):
    def __init__(self, args):
        super().__init__()
        self.args = args
        self.n_agents = args.n_agents
        self.state_dim = int(np.prod(args.state_shape))
        self.embed_dim = args.mixing_embed_dim
        dev = getattr(args, "device", "cpu")
        layers = getattr(args, "hypernet_layers", 1)
        self.hypernet_layers = layers
        S, E, N = self.state_dim, self.embed_dim, self.n_agents
        if layers == 1:
            self.hyper_w_1 = nn.Linear(S, E * N, device=dev)
            self.hyper_w_final = nn.Linear(S, E, device=dev)
        elif layers == 2:
            HE = args.hypernet_embed
            self.hyper_w_1 = nn.Sequential(nn.Linear(S, HE, device=dev), nn.ReLU(), nn.Linear(HE, E * N, device=dev))
            self.hyper_w_final = nn.Sequential(nn.Linear(S, HE, device=dev), nn.ReLU(), nn.Linear(HE, E, device=dev))
        elif layers > 2:
            raise Exception("Sorry >2 hypernet layers is not implemented!")
        else:
            raise Exception("Error setting number of hypernet layers.")
        self.hyper_b_1 = nn.Linear(S, E, device=dev)
        self.V = nn.Sequential(nn.Linear(S, E, device=dev), nn.ReLU(), nn.Linear(E, 1, device=dev))

    def _cparams(self):
        if self.hypernet_layers == 2:
            w1 = [self.hyper_w_1[0].weight, self.hyper_w_1[0].bias, self.hyper_w_1[2].weight, self.hyper_w_1[2].bias]
            wf = [self.hyper_w_final[0].weight, self.hyper_w_final[0].bias, self.hyper_w_final[2].weight,
                  self.hyper_w_final[2].bias]
            he = self.args.hypernet_embed
        else:
            w1 = [self.hyper_w_1.weight, self.hyper_w_1.bias, None, None]
            wf = [self.hyper_w_final.weight, self.hyper_w_final.bias, None, None]
            he = 0
        ts = w1 + wf + [self.hyper_b_1.weight, self.hyper_b_1.bias, self.V[0].weight, self.V[0].bias,
                        self.V[2].weight, self.V[2].bias]
        keep = [None if t is None else t.detach().float().contiguous() for t in ts]
        p = _native.MlgQMixParams(*[None if t is None else _native.ptr(t) for t in keep],
                                  self.n_agents, self.state_dim, self.embed_dim, he, self.hypernet_layers)
        return p, keep

    def forward(self, agent_qs, states):
        bs = agent_qs.size(0)
        qs = agent_qs.reshape(-1, self.n_agents).float().contiguous()
        st = states.reshape(-1, self.state_dim).float().contiguous()
        p, keep = self._cparams()
        from ...ops import qmix_forward
        empty = qs.new_empty(0)
        out = qmix_forward([empty if t is None else t for t in keep], qs, st,
                           [p.n_agents, p.state_dim, p.embed_dim, p.hypernet_embed, p.hypernet_layers])
        return out.view(bs, -1, 1)
