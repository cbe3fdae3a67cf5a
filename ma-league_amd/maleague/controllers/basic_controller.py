"""Parameter-shared multi-agent controller (API of src/marl/controllers/basic_controller.py:12-101).

forward(ep_batch, t) builds the agent inputs [obs_t | onehot(a_{t-1}) | agent id] and runs the DRQN
cell in one fused gfx950 kernel (mlg_mac_forward); the input concatenation is never materialised.
"""
from __future__ import annotations

from typing import OrderedDict

import torch

from .. import _native
from ..components.action_selectors import REGISTRY as action_REGISTRY
from ..components.batch_view import mlg_batch
from ..exceptions import HiddenStateNotInitialized
from ..modules.agents import REGISTRY as agent_REGISTRY
from ..utils.checkpoint import save_module


class MultiAgentController:
    def __init__(self, scheme, groups, args):
        self.n_agents = args.n_agents
        self.n_actions = args.n_actions
        self.args = args
        self.input_shape = self._get_input_shape(scheme)
        self.agent = self._build_agent(self.input_shape)
        self.agent_output_type = args.agent_output_type
        self.action_selector = action_REGISTRY[args.action_selector](args)
        self.hidden_states = None
        self.agent.trained_steps = 0
        if getattr(args, "freeze_native", False):
            for p in self.agent.parameters():
                p.requires_grad = False

    def _build_agent(self, input_shape):
        raise NotImplementedError()

    def _get_input_shape(self, scheme):
        raise NotImplementedError()


class BasicMAC(MultiAgentController):
    def select_actions(self, ep_batch, t_ep, t_env, bs=slice(None), test_mode=False):
        avail_actions = ep_batch["avail_actions"][:, t_ep]
        agent_outs = self.forward(ep_batch, t_ep, test_mode=test_mode)
        return self.action_selector.select(agent_outs[bs], avail_actions[bs], t_env, test_mode)

    def forward(self, ep_batch, t, test_mode=False):
        if self.agent_output_type != "q":
            raise NotImplementedError("pi_logits output (COMA) is out of scope for this build")
        if self.hidden_states is None:
            raise HiddenStateNotInitialized()
        B, N, H = ep_batch.batch_size, self.n_agents, self.args.rnn_hidden_dim
        mb, keep = mlg_batch(ep_batch, required=("obs", "actions_onehot"))
        h_in = self.hidden_states.reshape(B * N, H).float().contiguous()
        q = torch.empty(B, N, self.n_actions, device=h_in.device)
        h_out = torch.empty(B * N, H, device=h_in.device)
        d = self.agent.dims()
        _native.call("mlg_mac_forward", _native.byref(d), _native.ptr(self.agent.packed()), _native.byref(mb), int(t),
                     _native.ptr(h_in), _native.ptr(q), _native.ptr(h_out), _native.stream_ptr())
        del keep
        self.hidden_states = h_out
        return q

    def update_trained_steps(self, update):
        self.agent.add_trained_steps(update)

    def init_hidden(self, batch_size):
        self.hidden_states = self.agent.init_hidden().unsqueeze(0).expand(batch_size, self.n_agents, -1)

    def parameters(self):
        return self.agent.parameters()

    def load_state(self, other_mac):
        self.agent.load_state_dict(other_mac.agent.state_dict())

    def load_state_dict(self, agent: OrderedDict):
        self.agent.load_state_dict(agent)

    def cuda(self):
        self.agent.cuda()

    def save_models(self, path, name):
        save_module(self.agent, f"{path}/{name}agent.th")

    def load_models(self, path, name):
        self.agent.load_state_dict(torch.load(f"{path}/{name}agent.th", map_location=lambda s, loc: s,
                                              weights_only=True))

    def _build_agent(self, input_shape):
        return agent_REGISTRY[self.args.agent](input_shape, self.args)

    def _get_input_shape(self, scheme):
        shape = scheme["obs"]["vshape"]
        if self.args.obs_last_action:
            shape += scheme["actions_onehot"]["vshape"][0]
        if self.args.obs_agent_id:
            shape += self.n_agents
        return shape
