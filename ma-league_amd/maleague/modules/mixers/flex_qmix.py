"""FlexQMixer / AttentionHyperNet (API + state_dict keys of src/marl/modules/mixers/flex_qmix.py:5-117).

Parameters live under the reference's names (``hyper_w_1``, ``hyper_w_final``, ``hyper_b_1``, ``V``; each
``fc1``, ``attn.in_trans``, ``attn.out_trans``, ``attn.scale_factor``, ``fc2``). The mixer runs inside the
REFIL learner pipeline (mlg_refil_train: hyper_fwd / mix_td / hyper_bwd kernels).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ... import _native
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

    def _dims(self):
        a = self.args
        return _native.MlgRefilDims(n_agents=a.n_agents, n_entities=a.n_entities, entity_shape=a.entity_shape,
                                    n_actions=a.n_actions, entity_last_action=int(bool(a.entity_last_action)),
                                    attn_embed_dim=a.hypernet_embed, attn_n_heads=a.attn_n_heads,
                                    rnn_hidden_dim=a.hypernet_embed)

    def forward(self, agent_qs, inputs, imagine_groups=None):
        """flex_qmix.py:73-117: agent_qs [bs, T, NA] (or [bs, T, 2 NA] with imagine_groups = (Wmask, Imask)
        [bs, T, NE, NE]); inputs = (entities [bs, T, NE, D0], entity_mask [bs, T, NE]) -> q_tot [bs, T, 1]."""
        entities, entity_mask = inputs
        bs, T, ne, d0 = entities.shape
        R = bs * T
        dev = entities.device
        d = self._dims()
        with torch.no_grad():
            flat = torch.cat([p.detach().float().reshape(-1) for p in self.parameters()])
            packed = torch.empty(_native.load().mlg_refil_packed_mixer_size(_native.byref(d)), device=dev)
        _native.call("mlg_refil_pack_mixer", _native.byref(d), _native.ptr(flat), _native.ptr(packed),
                     _native.stream_ptr())
        qs = agent_qs.reshape(R, -1).float().contiguous()
        ent = entities.reshape(R, ne, d0).float().contiguous()
        em = entity_mask.reshape(R, ne).to(torch.uint8).contiguous()
        wm = im = None
        if imagine_groups is not None:
            wm = imagine_groups[0].reshape(R, ne, ne).to(torch.uint8).contiguous()
            im = imagine_groups[1].reshape(R, ne, ne).to(torch.uint8).contiguous()
        from ...ops import refil_mixer_forward, struct_fields
        out = refil_mixer_forward(packed, qs, ent, em, wm, im, int(bool(self.args.softmax_mixing_weights)),
                                  struct_fields(d))
        return out.view(bs, T, 1)
