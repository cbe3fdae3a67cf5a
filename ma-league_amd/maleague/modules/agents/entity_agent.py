"""EntityAttentionRNNAgent / ImagineEntityAttentionRNNAgent (API + state_dict keys of
src/marl/modules/agents/entity_rnn_agent.py:8-126): fc1 -> EntityAttentionLayer -> fc2 -> GRUCell -> fc3.

Parameters are ordinary nn.Linear / nn.GRUCell tensors under the reference's names (``fc1``, ``attn.in_trans``,
``attn.out_trans``, ``attn.scale_factor``, ``fc2``, ``rnn``, ``fc3``). Compute runs in the gfx950 kernels from a
packed copy (mlg_refil_pack_agent) refreshed whenever a parameter changed: ``forward`` over (bs, ts) steps through
mlg_refil_agent_forward; the rollout (mlg_refil_rollout) and the learner (mlg_refil_train) fuse it.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ... import _native
from ...utils.flat import flat_view
from ..layers.attention import EntityAttentionLayer
from .drqn_agent import AgentNetwork


class EntityAttentionRNNAgent(AgentNetwork):
    def __init__(self, input_shape, args):
        super().__init__(input_shape, args)
        if getattr(args, "pooling_type", None) is not None:
            raise NotImplementedError("EntityPoolingLayer (pooling_type) is not built; REFIL uses attention")
        dev = getattr(args, "device", "cpu")
        E, H = args.attn_embed_dim, args.rnn_hidden_dim
        self.fc1 = nn.Linear(input_shape, E, device=dev)
        self.attn = EntityAttentionLayer(E, E, E, args)
        self.fc2 = nn.Linear(E, H, device=dev)
        self.rnn = nn.GRUCell(H, H, device=dev)
        self.fc3 = nn.Linear(H, args.n_actions, device=dev)
        self._packed = None
        self._packed_key = None
        self._dirty = 0

    # ---- kernel plumbing --------------------------------------------------------------------
    def dims(self) -> _native.MlgRefilDims:
        a = self.args
        la = bool(getattr(a, "entity_last_action", True))
        return _native.MlgRefilDims(n_agents=a.n_agents, n_entities=a.n_entities,
                                    entity_shape=self.input_shape - (a.n_actions if la else 0), n_actions=a.n_actions,
                                    entity_last_action=int(la), attn_embed_dim=a.attn_embed_dim,
                                    attn_n_heads=a.attn_n_heads, rnn_hidden_dim=a.rnn_hidden_dim)

    def mark_dirty(self):
        self._dirty += 1

    def flat_parameters(self) -> torch.Tensor:
        """named_parameters() concatenated (the canonical order the C ABI documents). When the parameters already are
        consecutive views of one fp32 buffer (a learner's FlatParams), that buffer itself: no copy, no launch."""
        params = list(self.parameters())
        flat = flat_view(params)
        if flat is not None:
            return flat
        with torch.no_grad():
            return torch.cat([p.detach().float().reshape(-1) for p in params])

    def packed(self) -> torch.Tensor:
        params = list(self.parameters())
        key = (self._dirty,) + tuple((p.data_ptr(), p._version) for p in params)
        if self._packed is None or key != self._packed_key:
            d = self.dims()
            n = _native.load().mlg_refil_packed_agent_size(_native.byref(d))
            if n < 0:
                raise _native.NativeError(_native.load().mlg_last_error().decode())
            dev = self.fc1.weight.device
            if self._packed is None or self._packed.numel() != n or self._packed.device != dev:
                self._packed = torch.empty(n, dtype=torch.float32, device=dev)
            flat = self.flat_parameters()
            _native.call("mlg_refil_pack_agent", _native.byref(d), _native.ptr(flat), _native.ptr(self._packed),
                         _native.stream_ptr())
            self._flat_keep = flat
            self._packed_key = key
        return self._packed

    def _load_from_state_dict(self, *args, **kwargs):
        super()._load_from_state_dict(*args, **kwargs)
        self.mark_dirty()

    # ---- reference API -------------------------------------------------------------------------
    def init_hidden(self):
        """A zero [1, H] state, cached per device (callers expand it and never write into it): no fill per run."""
        w = self.fc1.weight
        h0 = getattr(self, "_h0", None)
        if h0 is None or h0.device != w.device or h0.dtype != w.dtype:
            self._h0 = h0 = w.new_zeros(1, self.args.rnn_hidden_dim)
        return h0

    def forward(self, inputs, hidden_state, ret_attn_logits=None):
        """inputs = (entities [bs, ts, ne, ed], obs_mask [bs, ts, ne, ne], entity_mask [bs, ts, ne]);
        hidden_state [bs, na, H] -> (q [bs, ts, na, A] (0 for masked agents), hs [bs, ts, na, H])."""
        if ret_attn_logits is not None:
            raise NotImplementedError("ret_attn_logits is a diagnostic of the reference; not built")
        entities, obs_mask, entity_mask = inputs
        bs, ts, ne, ed = entities.shape
        na, H, A = self.args.n_agents, self.args.rnn_hidden_dim, self.args.n_actions
        dev = entities.device
        ent = entities.float().contiguous()
        om = obs_mask.to(torch.uint8).contiguous()
        em = entity_mask.to(torch.uint8).contiguous()
        h = hidden_state.reshape(bs, na, H).float().contiguous()
        q = torch.empty(bs, ts, na, A, device=dev)
        hs = torch.empty(bs, ts, na, H, device=dev)
        d = self.dims()
        P = self.packed()
        from ...ops import refil_agent_step, struct_fields
        dl = struct_fields(d)
        for t in range(ts):
            et, ot, mt = ent[:, t].contiguous(), om[:, t].contiguous(), em[:, t].contiguous()
            qt, ht = refil_agent_step(P, et, ot, mt, h, dl)
            q[:, t] = qt
            hs[:, t] = ht
            h = ht
        return q, hs


def entitymask2attnmask(entity_mask):
    """1 - (1 - m_i)(1 - m_j) (entity_rnn_agent.py:80-86)."""
    m = entity_mask.to(torch.bool)
    return (m.unsqueeze(-1) | m.unsqueeze(-2)).to(torch.uint8)


def imagine_masks(groupA, entity_mask, obs_mask):
    """The mask algebra of ImagineEntityAttentionRNNAgent.forward (entity_rnn_agent.py:93-118) for a given group
    draw groupA [bs, 1, ne] (uint8): returns the obs masks of the within / interact copies [bs, ts, ne, ne] and
    the mixer masks (W, I) without observability [bs, 1, ne, ne]. Integer mask work, host-side plumbing."""
    em0 = entity_mask[:, [0]].to(torch.bool)
    gA = groupA.to(torch.bool) | em0
    gB = (~groupA.to(torch.bool)) | em0
    A2 = gA.unsqueeze(-1) | gA.unsqueeze(-2)
    B2 = gB.unsqueeze(-1) | gB.unsqueeze(-2)
    interact = (~A2) | (~B2)
    within = ~interact
    active = em0.unsqueeze(-1) | em0.unsqueeze(-2)
    om = obs_mask.to(torch.bool)
    return ((within | om).to(torch.uint8), (interact | om).to(torch.uint8), (within | active).to(torch.uint8),
            (interact | active).to(torch.uint8))


class ImagineEntityAttentionRNNAgent(EntityAttentionRNNAgent):
    def forward(self, inputs, hidden_state, imagine=False, groupA=None, **kwargs):
        if not imagine:
            return super().forward(inputs, hidden_state)
        entities, obs_mask, entity_mask = inputs
        bs, ts, ne, _ = entities.shape
        if groupA is None:  # one random split of the entities per episode (entity_rnn_agent.py:95-97)
            p = torch.rand(bs, 1, 1, device=entities.device).repeat(1, 1, ne)
            groupA = torch.bernoulli(p).to(torch.uint8)
        within, interact, Wn, In = imagine_masks(groupA, entity_mask, obs_mask)
        q, h = super().forward((entities.repeat(3, 1, 1, 1),
                                torch.cat([obs_mask.to(torch.uint8), within, interact], dim=0),
                                entity_mask.repeat(3, 1, 1)), hidden_state.repeat(3, 1, 1))
        return q, h, (Wn.repeat(1, ts, 1, 1), In.repeat(1, ts, 1, 1))
