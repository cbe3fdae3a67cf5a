"""``torch.ops.maleague.*``: the stand-alone hot-path ops as PyTorch custom operators (the plugin
classes call the HIP library through ops PyTorch can see, next to the plain C ABI for non-torch callers).

Each op is registered with ``torch.library.custom_op`` (functional: it allocates its outputs) and a fake
(meta) implementation giving the output shapes, so ``torch.compile`` / graph capture treat it as one opaque node
instead of breaking the graph at a ctypes call. The implementation enqueues the ``libmaleague.so`` entry point
(include/maleague.h) on the current HIP stream of the inputs' device. There is no CPU implementation: the ops
raise on host tensors like every product path.

| op                                   | C ABI entry point         | reference                                           |
|--------------------------------------|---------------------------|-----------------------------------------------------|
| ``maleague::agent_forward``          | ``mlg_agent_forward``     | DRQNAgentNetwork.forward (drqn_agent.py:29-35)     |
| ``maleague::select_actions``         | ``mlg_select_actions``    | EpsilonGreedyActionSelector.select (action_selectors.py:44-62) |
| ``maleague::qmix_forward``           | ``mlg_qmix_forward``      | QMixer.forward (qmix.py:41-59)                      |
| ``maleague::refil_attention``        | ``mlg_refil_attention``   | EntityAttentionLayer.forward (attention.py:24-79)   |
| ``maleague::refil_mixer_forward``    | ``mlg_refil_mixer_forward`` | FlexQMixer.forward (flex_qmix.py:73-117)          |
| ``maleague::refil_agent_step``       | ``mlg_refil_agent_forward`` | EntityAttentionRNNAgent.forward, one step (entity_rnn_agent.py:32-65) |

The rollout and learner entry points (``mlg_rollout*``, ``mlg_qlearner_train``, ``mlg_refil_train``) take the
replay ring, env state and optimizer state as in-place structs and stay direct calls of the stepper / learner
classes.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
from torch import Tensor
from torch.library import custom_op, register_fake

from . import _native


def struct_fields(s) -> List[int]:
    """A ctypes dims struct (MlgAgentDims, MlgRefilDims, ...) as the int list the ops take."""
    return [int(getattr(s, f)) for f, _ in s._fields_]


def _stream(t: Tensor) -> int:
    return _native.stream_ptr(t.device)


def _opt(t: Optional[Tensor]):
    return None if t is None or t.numel() == 0 else _native.ptr(t)


# ---- DRQNAgentNetwork.forward ------------------------------------------------------------------------------
@custom_op("maleague::agent_forward", mutates_args=())
def agent_forward(packed: Tensor, inputs: Tensor, h_in: Tensor, dims: List[int]) -> Tuple[Tensor, Tensor]:
    """dims = [d_obs, n_actions, n_agents, hidden, d_in, obs_last_action, obs_agent_id] (MlgAgentDims);
    inputs [R, d_in], h_in [R, H] -> (q [R, A], h_out [R, H])."""
    d = _native.MlgAgentDims(*[int(v) for v in dims])
    R = inputs.shape[0]
    q = inputs.new_empty(R, d.n_actions)
    h_out = inputs.new_empty(R, d.hidden)
    _native.call("mlg_agent_forward", _native.byref(d), _native.ptr(packed), _native.ptr(inputs), _native.ptr(h_in),
                 _native.ptr(q), _native.ptr(h_out), R, _stream(inputs))
    return q, h_out


@register_fake("maleague::agent_forward")
def _agent_forward_fake(packed, inputs, h_in, dims):
    R = inputs.shape[0]
    return inputs.new_empty(R, dims[1]), inputs.new_empty(R, dims[3])


# ---- EpsilonGreedyActionSelector.select ----------------------------------------------------------------------
@custom_op("maleague::select_actions", mutates_args=())
def select_actions(q: Tensor, avail: Tensor, keys: Tensor, episodes: Tensor, t: int, epsilon: float
                   ) -> Tuple[Tensor, Tensor]:
    """q [B, N, A] f32, avail [B, N, A] int32, keys [B] int64 (counter-RNG key per env), episodes [B] int32 ->
    (actions [B, N] int64, is_greedy [B, N] int64)."""
    B, N, A = q.shape
    actions = torch.empty(B, N, dtype=torch.int64, device=q.device)
    greedy = torch.empty(B, N, dtype=torch.int64, device=q.device)
    _native.call("mlg_select_actions", _native.ptr(q), _native.ptr(avail), B * N, A, N, _native.ptr(keys),
                 _native.ptr(episodes), int(t), float(epsilon), _native.ptr(actions), _native.ptr(greedy), _stream(q))
    return actions, greedy


@register_fake("maleague::select_actions")
def _select_actions_fake(q, avail, keys, episodes, t, epsilon):
    B, N, _ = q.shape
    return q.new_empty(B, N, dtype=torch.int64), q.new_empty(B, N, dtype=torch.int64)


# ---- QMixer.forward ------------------------------------------------------------------------------------------
@custom_op("maleague::qmix_forward", mutates_args=())
def qmix_forward(params: List[Tensor], agent_qs: Tensor, states: Tensor, dims: List[int]) -> Tensor:
    """params = the 14 MlgQMixParams tensors in header order (zero-size for the absent second layers of a
    one-layer hypernet); dims = [n_agents, state_dim, embed_dim, hypernet_embed, hypernet_layers]; agent_qs [R, N],
    states [R, S] -> q_tot [R]."""
    p = _native.MlgQMixParams(*[_opt(t) for t in params], *[int(v) for v in dims])
    out = agent_qs.new_empty(agent_qs.shape[0])
    _native.call("mlg_qmix_forward", _native.byref(p), _native.ptr(agent_qs), _native.ptr(states), _native.ptr(out),
                 agent_qs.shape[0], _stream(agent_qs))
    return out


@register_fake("maleague::qmix_forward")
def _qmix_forward_fake(params, agent_qs, states, dims):
    return agent_qs.new_empty(agent_qs.shape[0])


# ---- EntityAttentionLayer.forward ----------------------------------------------------------------------------
@custom_op("maleague::refil_attention", mutates_args=())
def refil_attention(w_in: Tensor, w_out: Tensor, b_out: Tensor, x: Tensor, pre_mask: Tensor, post_mask: Tensor,
                    n_heads: int) -> Tensor:
    """x [bs, ne, in], pre_mask [bs, nq, ne] u8, post_mask [bs, nq] u8 -> y [bs, nq, out]."""
    bs, ne, _ = x.shape
    nq = post_mask.shape[1]
    y = x.new_empty(bs, nq, w_out.shape[0])
    _native.call("mlg_refil_attention", _native.ptr(w_in), _native.ptr(w_out), _native.ptr(b_out), _native.ptr(x),
                 _native.ptr(pre_mask), _native.ptr(post_mask), int(bs), int(ne), int(nq), int(n_heads),
                 _native.ptr(y), None, None, None, None, None, _stream(x))
    return y


@register_fake("maleague::refil_attention")
def _refil_attention_fake(w_in, w_out, b_out, x, pre_mask, post_mask, n_heads):
    return x.new_empty(x.shape[0], post_mask.shape[1], w_out.shape[0])


def _refil_dims(dims):
    return _native.MlgRefilDims(*[int(v) for v in dims])


# ---- FlexQMixer.forward --------------------------------------------------------------------------------------
@custom_op("maleague::refil_mixer_forward", mutates_args=())
def refil_mixer_forward(packed: Tensor, agent_qs: Tensor, entities: Tensor, entity_mask: Tensor,
                        w_mask: Optional[Tensor], i_mask: Optional[Tensor], softmax_mixing_weights: int,
                        dims: List[int]) -> Tensor:
    """dims = MlgRefilDims fields; agent_qs [R, NA] (or [R, 2 NA] with both imagine masks [R, NE, NE]),
    entities [R, NE, D0], entity_mask [R, NE] -> q_tot [R]."""
    d = _refil_dims(dims)
    R = agent_qs.shape[0]
    out = agent_qs.new_empty(R)
    _native.call("mlg_refil_mixer_forward", _native.byref(d), _native.ptr(packed), _native.ptr(agent_qs),
                 _native.ptr(entities), _native.ptr(entity_mask), _opt(w_mask), _opt(i_mask),
                 int(softmax_mixing_weights), _native.ptr(out), R, _stream(agent_qs))
    return out


@register_fake("maleague::refil_mixer_forward")
def _refil_mixer_forward_fake(packed, agent_qs, entities, entity_mask, w_mask, i_mask, softmax_mixing_weights, dims):
    return agent_qs.new_empty(agent_qs.shape[0])


# ---- EntityAttentionRNNAgent.forward, one step ---------------------------------------------------------------
@custom_op("maleague::refil_agent_step", mutates_args=())
def refil_agent_step(packed: Tensor, entities: Tensor, obs_mask: Tensor, entity_mask: Tensor, h_in: Tensor,
                     dims: List[int]) -> Tuple[Tensor, Tensor]:
    """entities [R, NE, D0], obs_mask [R, NE, NE] u8, entity_mask [R, NE] u8, h_in [R, NA, H] ->
    (q [R, NA, A], h_out [R, NA, H])."""
    d = _refil_dims(dims)
    R = entities.shape[0]
    q = entities.new_empty(R, d.n_agents, d.n_actions)
    h = entities.new_empty(R, d.n_agents, d.rnn_hidden_dim)
    _native.call("mlg_refil_agent_forward", _native.byref(d), _native.ptr(packed), _native.ptr(entities),
                 _native.ptr(obs_mask), _native.ptr(entity_mask), _native.ptr(h_in), _native.ptr(q), _native.ptr(h),
                 int(R), _stream(entities))
    return q, h


@register_fake("maleague::refil_agent_step")
def _refil_agent_step_fake(packed, entities, obs_mask, entity_mask, h_in, dims):
    R = entities.shape[0]
    return entities.new_empty(R, dims[0], dims[3]), entities.new_empty(R, dims[0], dims[7])


OPS = ("agent_forward", "select_actions", "qmix_forward", "refil_attention", "refil_mixer_forward",
       "refil_agent_step")
