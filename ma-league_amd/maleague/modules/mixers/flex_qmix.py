"""FlexQMixer / AttentionHyperNet (API + state_dict keys of src/marl/modules/mixers/flex_qmix.py:5-117).

Parameters live under the reference's names (``hyper_w_1``, ``hyper_w_final``, ``hyper_b_1``, ``V``; each
``fc1``, ``attn.in_trans``, ``attn.out_trans``, ``attn.scale_factor``, ``fc2``). The mixer runs inside the
REFIL learner pipeline (mlg_refil_train: hyper_fwd / mix_td / hyper_bwd kernels).
"""
from __future__ import annotations

import torch.nn as nn

from ..layers.attention import EntityAttentionLayer


class AttentionHyperNet(nn.Module):
    def __init__(self, args, extra_dims=0, mode="matrix"):
        super().__init__()
        if getattr(args, "pooling_type", None) is not None:
            raise NotImplementedError("EntityPoolingLayer (pooling_type) is not built; REFIL uses attention")
        self.args = args
        self.mode = mode
        self.entity_dim = args.entity_shape + (args.n_actions if args.entity_last_action else 0) + extra_dims
        dev = getattr(args, "device", "cpu")
        he = args.hypernet_embed
        self.fc1 = nn.Linear(self.entity_dim, he, device=dev)
        self.attn = EntityAttentionLayer(he, he, he, args)
        self.fc2 = nn.Linear(he, args.mixing_embed_dim, device=dev)


class FlexQMixer(nn.Module):
    def __init__(self, args):
        super().__init__()
        self.args = args
        self.n_agents = args.n_agents
        self.embed_dim = args.mixing_embed_dim
        self.hyper_w_1 = AttentionHyperNet(args, mode="matrix")
        self.hyper_w_final = AttentionHyperNet(args, mode="vector")
        self.hyper_b_1 = AttentionHyperNet(args, mode="vector")
        self.V = AttentionHyperNet(args, mode="scalar")
        if getattr(args, "mixer_non_lin", "elu") != "elu":
            raise NotImplementedError("mixer_non_lin: only elu (the default) is built")
