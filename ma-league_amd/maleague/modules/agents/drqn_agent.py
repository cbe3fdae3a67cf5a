"""DRQN agent: fc1 -> ReLU -> GRUCell -> fc2 (API + state_dict keys of src/marl/modules/agents/drqn_agent.py:7-35).

Parameters are ordinary nn.Linear / nn.GRUCell tensors (so ``{name}agent.th`` checkpoints interoperate with
the reference); the forward pass runs in the gfx950 kernel (mlg_agent_forward) from a packed copy of the
weights that is refreshed whenever the parameters change.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ... import _native


class AgentNetwork(nn.Module):
    def __init__(self, input_shape, args):
        super().__init__()
        self.args = args
        self.input_shape = input_shape
        self._trained_host = 0
        self._trained_dev = None  # device-side running count (no host sync per train step)
        self.trained_steps = 0

    @property
    def trained_steps(self) -> int:
        """Agent.trained_steps (agent_network.py:15): env steps trained on; device counts resolve on read."""
        extra = 0 if self._trained_dev is None else int(round(float(self._trained_dev.item())))
        return self._trained_host + extra

    @trained_steps.setter
    def trained_steps(self, value: int):
        self._trained_host = int(value)
        self._trained_dev = None

    def trained_steps_with(self, device_count: float) -> int:
        """trained_steps given the device counter's value read elsewhere (no extra device round trip)."""
        return self._trained_host + int(round(float(device_count)))

    def trained_counter(self, device) -> torch.Tensor:
        """The device-side float64 running count a learner kernel adds to (created at 0 on first use)."""
        if self._trained_dev is None or self._trained_dev.device != torch.device(device):
            extra = 0.0 if self._trained_dev is None else float(self._trained_dev.item())
            self._trained_dev = torch.full((), extra, dtype=torch.float64, device=device)
        return self._trained_dev

    def add_trained_steps(self, update):
        if torch.is_tensor(update):
            if self._trained_dev is None:
                self._trained_dev = update.detach().to(torch.float64).clone()
            else:
                self._trained_dev.add_(update.detach())
        else:
            self._trained_host += int(update)

    def init_hidden(self):
        raise NotImplementedError()

    def forward(self, inputs, hidden_state):
        raise NotImplementedError()

    def count_parameters(self):
        return sum(p.numel() for p in self.parameters() if p.requires_grad)


class DRQNAgentNetwork(AgentNetwork):
    def __init__(self, input_shape, args):
        super().__init__(input_shape, args)
        dev = getattr(args, "device", "cpu")
        self.fc1 = nn.Linear(input_shape, args.rnn_hidden_dim, device=dev)
        self.gru = nn.GRUCell(args.rnn_hidden_dim, args.rnn_hidden_dim, device=dev)
        self.fc2 = nn.Linear(args.rnn_hidden_dim, args.n_actions, device=dev)
        self._packed = None
        self._packed_key = None
        self._dirty = 0
        self._h0 = None

    # ---- kernel plumbing --------------------------------------------------------------------
    def dims(self) -> _native.MlgAgentDims:
        a = self.args
        return _native.MlgAgentDims(d_obs=self.input_shape - (a.n_actions if a.obs_last_action else 0)
                                    - (a.n_agents if a.obs_agent_id else 0),
                                    n_actions=a.n_actions, n_agents=a.n_agents, hidden=a.rnn_hidden_dim,
                                    d_in=self.input_shape, obs_last_action=int(bool(a.obs_last_action)),
                                    obs_agent_id=int(bool(a.obs_agent_id)))

    def mark_dirty(self):
        """Call after parameters were modified outside torch (e.g. by the fused optimizer kernel)."""
        self._dirty += 1

    def packed(self) -> torch.Tensor:
        """Packed weight block (agent_device.h layout); rebuilt when any parameter changed."""
        params = [self.fc1.weight, self.fc1.bias, self.gru.weight_ih, self.gru.bias_ih, self.gru.weight_hh,
                  self.gru.bias_hh, self.fc2.weight, self.fc2.bias]
        key = (self._dirty,) + tuple((p.data_ptr(), p._version) for p in params)
        if self._packed is None or key != self._packed_key:
            d = self.dims()
            n = _native.load().mlg_packed_agent_size(_native.byref(d))
            if n < 0:
                raise _native.NativeError(_native.load().mlg_last_error().decode())
            dev = self.fc1.weight.device
            if self._packed is None or self._packed.numel() != n or self._packed.device != dev:
                self._packed = torch.empty(n, dtype=torch.float32, device=dev)
            with torch.no_grad():
                cp = [p.detach().float().contiguous() for p in params]
            cparams = _native.MlgAgentParams(*[_native.ptr(p) for p in cp])
            _native.call("mlg_pack_agent", _native.byref(d), _native.byref(cparams), _native.ptr(self._packed),
                         _native.stream_ptr())
            self._packed_key = key
        return self._packed

    def _load_from_state_dict(self, *args, **kwargs):
        super()._load_from_state_dict(*args, **kwargs)
        self.mark_dirty()

    # ---- reference API -------------------------------------------------------------------------
    def init_hidden(self):
        """A zero [1, H] state; one cached tensor per device (callers expand it and never write into it), so a
        rollout's MAC reset launches no fill."""
        w = self.fc1.weight
        if self._h0 is None or self._h0.device != w.device or self._h0.dtype != w.dtype:
            self._h0 = w.new_zeros(1, self.args.rnn_hidden_dim)
        return self._h0

    def forward(self, inputs, hidden_state):
        H = self.args.rnn_hidden_dim
        x = inputs.float().contiguous()
        h_in = hidden_state.reshape(-1, H).float().contiguous()
        from ...ops import struct_fields
        return torch.ops.maleague.agent_forward(self.packed(), x, h_in, struct_fields(self.dims()))
