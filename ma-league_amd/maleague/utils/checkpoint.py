"""Checkpoint writing in the reference's file format (q_learner.py:133-137, basic_controller.py:68-69).

The learners keep parameters and RMSprop state as views into flat fp32 buffers. torch.save of a view stores
its whole underlying storage, so a state dict is cloned tensor by tensor first: each file then holds exactly
the tensors the reference's would (same keys, shapes, dtypes, one storage per tensor)."""
from __future__ import annotations

from collections import OrderedDict

import torch


def _own(v):
    return v.detach().clone() if isinstance(v, torch.Tensor) else v


def module_state(module) -> OrderedDict:
    return OrderedDict((k, _own(v)) for k, v in module.state_dict().items())


def optimizer_state(optimiser) -> dict:
    sd = optimiser.state_dict()
    return {"state": {i: {k: _own(v) for k, v in st.items()} for i, st in sd["state"].items()},
            "param_groups": sd["param_groups"]}


def save_module(module, path):
    torch.save(module_state(module), path)


def save_optimizer(optimiser, path):
    torch.save(optimizer_state(optimiser), path)
