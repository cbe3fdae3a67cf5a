"""VDN mixer (src/marl/modules/mixers/vdn.py:5-9)."""
import torch
import torch.nn as nn


class VDNMixer(nn.Module):
    def forward(self, agent_qs, batch):
        return torch.sum(agent_qs, dim=2, keepdim=True)
