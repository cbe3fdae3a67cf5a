"""EntityMAC (API of src/marl/controllers/entity_controller.py:7-36): BasicMAC over entity inputs.

Inputs per step: entities [bs, ts, ne, ed] with the last action one-hot appended to the agent entities
(entity_last_action; zeros at t = 0), obs_mask, entity_mask. ``t`` may be an int (one step, the rollout case,
-> [B, N, A]), a slice, or None = the whole episode (the learner case, refil_learner.py:123,149 ->
[B, T, N, A]); the reference only serves slices starting at 0 with a consistent stop, these are the
intended semantics. The fused rollout (mlg_refil_rollout) runs this MAC inside the kernel.
"""
from __future__ import annotations

import torch

from .basic_controller import BasicMAC
from ..exceptions import HiddenStateNotInitialized


class EntityMAC(BasicMAC):
    def _as_slice(self, batch, t):
        if t is None:
            return slice(0, batch.max_seq_length)
        if isinstance(t, int):
            return slice(t, t + 1)
        return slice(t.start or 0, batch.max_seq_length if t.stop is None else t.stop)

    def _build_inputs(self, batch, t):
        t = self._as_slice(batch, t)
        ents = batch["entities"][:, t]
        bs, ts, ne, _ = ents.shape
        parts = [ents]
        if self.args.entity_last_action:
            acs = torch.zeros(bs, ts, ne, self.args.n_actions, device=ents.device, dtype=ents.dtype)
            if t.start == 0:
                acs[:, 1:, :self.args.n_agents] = batch["actions_onehot"][:, slice(0, t.stop - 1)]
            else:
                acs[:, :, :self.args.n_agents] = batch["actions_onehot"][:, slice(t.start - 1, t.stop - 1)]
            parts.append(acs)
        return torch.cat(parts, dim=3), batch["obs_mask"][:, t], batch["entity_mask"][:, t]

    def forward(self, ep_batch, t, test_mode=False, imagine=False, groupA=None):
        if self.agent_output_type != "q":
            raise NotImplementedError("pi_logits output is out of scope for this build")
        if self.hidden_states is None:
            raise HiddenStateNotInitialized()
        inputs = self._build_inputs(ep_batch, t)
        if imagine:
            q, hs, groups = self.agent(inputs, self.hidden_states, imagine=True, groupA=groupA)
            self.hidden_states = hs[:, -1]
            return q, groups
        q, hs = self.agent(inputs, self.hidden_states)
        self.hidden_states = hs[:, -1]
        if isinstance(t, int):
            return q[:, 0]
        return q

    def _get_input_shape(self, scheme):
        shape = scheme["entities"]["vshape"][-1]
        if self.args.entity_last_action:
            shape += scheme["actions_onehot"]["vshape"][0]
        return shape
