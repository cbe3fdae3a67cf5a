"""EntityAttentionLayer (API + state_dict keys of src/marl/modules/layers/attention.py:7-79).

Parameters and the ``scale_factor`` buffer are those of the reference (``in_trans.weight`` [3E, in],
``out_trans.weight`` [out, E], ``out_trans.bias``), so REFIL checkpoints interoperate. The computation runs
inside the REFIL kernels (refil_device.h attn_fwd / attn_bwd); ``forward`` calls mlg_refil_attention.
"""
from __future__ import annotations

import torch
import torch.nn as nn



class EntityAttentionLayer(nn.Module):
    def __init__(self, in_dim, embed_dim, out_dim, args):
        super().__init__()
        self.in_dim, self.embed_dim, self.out_dim = in_dim, embed_dim, out_dim
        self.n_heads = args.attn_n_heads
        self.n_agents = args.n_agents
        self.args = args
        assert self.embed_dim % self.n_heads == 0, "Embed dim must be divisible by n_heads"
        self.head_dim = self.embed_dim // self.n_heads
        dev = getattr(args, "device", "cpu")
        self.register_buffer("scale_factor", torch.scalar_tensor(self.head_dim, device=dev).sqrt())
        self.in_trans = nn.Linear(self.in_dim, self.embed_dim * 3, bias=False, device=dev)
        self.out_trans = nn.Linear(self.embed_dim, self.out_dim, device=dev)

    def forward(self, entities, pre_mask=None, post_mask=None, ret_attn_logits=None):
        """entities [bs, ne, in]; pre_mask [bs, >=nq, >=ne] (True/1 = masked); post_mask [bs, nq] -> [bs, nq, out]."""
        if ret_attn_logits is not None:
            raise NotImplementedError("ret_attn_logits is a diagnostic of the reference; not built")
        bs, ne, _ = entities.shape
        nq = post_mask.shape[1]
        dev = entities.device
        x = entities.float().contiguous()
        pre = pre_mask[:, :nq, :ne].to(torch.uint8).contiguous()
        post = post_mask.to(torch.uint8).contiguous()
        w_in = self.in_trans.weight.detach().float().contiguous()
        w_out = self.out_trans.weight.detach().float().contiguous()
        b_out = self.out_trans.bias.detach().float().contiguous()
        from ...ops import refil_attention
        return refil_attention(w_in, w_out, b_out, x, pre, post, int(self.n_heads))
