"""ctypes binding of libmaleague.so, the C ABI declared in include/maleague.h.

The HIP library is the product path: every op of the hot path calls into it. There is no CPU
fallback -- if the library is missing or no GPU is present, calls raise loudly.
Tensors cross the boundary as raw device pointers (``tensor.data_ptr()``) plus sizes; kernels run
on the caller's current HIP stream (``torch.cuda.current_stream().cuda_stream``).
"""
from __future__ import annotations

import ctypes
import os

import torch

MAXU = 64
_LIB_PATH = os.environ.get("MLG_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib",
                                                      "libmaleague.so")


class NativeError(RuntimeError):
    """Raised when a libmaleague call fails (the C side's mlg_last_error())."""


class MlgEnvSpec(ctypes.Structure):
    _fields_ = [("U", ctypes.c_int32), ("n_agents", ctypes.c_int32), ("n_actions", ctypes.c_int32),
                ("grid", ctypes.c_int32), ("episode_limit", ctypes.c_int32), ("stochastic", ctypes.c_int32),
                ("policy_team", ctypes.c_int32), ("n_policy_teams", ctypes.c_int32),
                ("team", ctypes.c_int32 * MAXU), ("role", ctypes.c_int32 * MAXU), ("melee", ctypes.c_int32 * MAXU),
                ("agent_unit", ctypes.c_int32 * MAXU), ("scripted", ctypes.c_int32 * 2), ("seed", ctypes.c_uint64)]


class MlgEnvState(ctypes.Structure):
    _fields_ = [("x", ctypes.c_void_p), ("y", ctypes.c_void_p), ("hp", ctypes.c_void_p), ("t", ctypes.c_void_p),
                ("episode", ctypes.c_void_p), ("B", ctypes.c_int32)]


class MlgBatch(ctypes.Structure):
    _fields_ = [("state", ctypes.c_void_p), ("obs", ctypes.c_void_p), ("actions", ctypes.c_void_p),
                ("avail", ctypes.c_void_p), ("reward", ctypes.c_void_p), ("terminated", ctypes.c_void_p),
                ("actions_onehot", ctypes.c_void_p), ("filled", ctypes.c_void_p), ("B", ctypes.c_int32),
                ("T1", ctypes.c_int32), ("ring_slot0", ctypes.c_int32), ("ring_size", ctypes.c_int32),
                ("full_write", ctypes.c_int32), ("rows", ctypes.c_void_p), ("slot_extent", ctypes.c_void_p)]


class MlgRunInfo(ctypes.Structure):
    _fields_ = [("ep_len", ctypes.c_void_p), ("ret", ctypes.c_void_p), ("won", ctypes.c_void_p),
                ("draw", ctypes.c_void_p), ("agent_rows", ctypes.c_void_p), ("ret_away", ctypes.c_void_p)]


class MlgAgentParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ["fc1_w", "fc1_b", "w_ih", "b_ih", "w_hh", "b_hh", "fc2_w", "fc2_b"]]


class MlgAgentDims(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ["d_obs", "n_actions", "n_agents", "hidden", "d_in", "obs_last_action",
                                              "obs_agent_id"]]


class MlgQMixParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ["hw1_0w", "hw1_0b", "hw1_2w", "hw1_2b", "hwf_0w", "hwf_0b", "hwf_2w",
                                              "hwf_2b", "hb1_w", "hb1_b", "v0_w", "v0_b", "v2_w", "v2_b"]] + \
               [(n, ctypes.c_int32) for n in ["n_agents", "state_dim", "embed_dim", "hypernet_embed",
                                              "hypernet_layers"]]


class MlgLearnerCfg(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ["B", "T", "N", "A", "d_obs", "H", "S", "E", "HE", "hypernet_layers",
                                              "mixer", "double_q", "obs_last_action", "obs_agent_id"]] + \
               [(n, ctypes.c_float) for n in ["gamma", "lr", "optim_alpha", "optim_eps", "grad_norm_clip"]]


class MlgLearnerBufs(ctypes.Structure):
    _fields_ = [("batch", MlgBatch)] + [(n, ctypes.c_void_p) for n in ["params", "grads", "square_avg",
                                                                      "target_params", "workspace", "stats",
                                                                      "target_sync", "trained_steps", "host_rows"]]


class MlgEntityEnvSpec(ctypes.Structure):
    _fields_ = [("base", MlgEnvSpec), ("min_agents", ctypes.c_int32), ("max_agents", ctypes.c_int32)]


class MlgEntityBatch(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ["entities", "obs_mask", "entity_mask", "actions", "avail", "reward",
                                              "terminated", "actions_onehot", "filled"]] + \
               [(n, ctypes.c_int32) for n in ["B", "T1", "ring_slot0", "ring_size", "full_write"]] + \
               [("rows", ctypes.c_void_p), ("slot_extent", ctypes.c_void_p)]


class MlgRefilDims(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ["n_agents", "n_entities", "entity_shape", "n_actions",
                                              "entity_last_action", "attn_embed_dim", "attn_n_heads",
                                              "rnn_hidden_dim"]]



class MlgRefilLearnerCfg(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ["B", "T", "n_agents", "n_entities", "entity_shape", "n_actions",
                                              "entity_last_action", "attn_embed_dim", "attn_n_heads", "rnn_hidden_dim",
                                              "hypernet_embed", "mixing_embed_dim", "double_q",
                                              "softmax_mixing_weights", "imagine"]] + \
               [(n, ctypes.c_float) for n in ["gamma", "lmbda", "lr", "optim_alpha", "optim_eps", "grad_norm_clip"]]


class MlgRefilLearnerBufs(ctypes.Structure):
    _fields_ = [("batch", MlgEntityBatch)] + [(n, ctypes.c_void_p) for n in ["groupA", "params", "grads", "square_avg",
                                                                           "target_params", "workspace", "stats",
                                                                           "trained_steps", "target_sync",
                                                                           "host_rows"]]


_P = ctypes.c_void_p
_I = ctypes.c_int32
# name -> (restype, argtypes); mirrors include/maleague.h one for one.
SIGNATURES = {
    "mlg_packed_agent_size": (ctypes.c_int64, [_P]),
    "mlg_pack_agent": (ctypes.c_int, [_P, _P, _P, _P]),
    "mlg_env_reset": (ctypes.c_int, [_P, _P, _P]),
    "mlg_env_step": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P, _P]),
    "mlg_env_observe": (ctypes.c_int, [_P, _P, _P, _P, _P, _P]),
    "mlg_rollout": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, ctypes.c_float, _I, _P]),
    "mlg_rollout_selfplay": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P, _P, ctypes.c_float, ctypes.c_float, _I, _P]),
    "mlg_agent_forward": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _I, _P]),
    "mlg_mac_forward": (ctypes.c_int, [_P, _P, _P, _I, _P, _P, _P, _P]),
    "mlg_select_actions": (ctypes.c_int, [_P, _P, _I, _I, _I, _P, _P, _I, ctypes.c_float, _P, _P, _P]),
    "mlg_qmix_forward": (ctypes.c_int, [_P, _P, _P, _P, _I, _P]),
    "mlg_qlearner_param_counts": (ctypes.c_int64, [_P, _P, _P]),
    "mlg_qlearner_workspace_floats": (ctypes.c_int64, [_P]),
    "mlg_qlearner_inline_rows": (ctypes.c_int, []),
    "mlg_qlearner_train": (ctypes.c_int, [_P, _P, _P]),
    "mlg_zero_slots_bytes": (ctypes.c_int, [_P, _P, _I, _I, _I, _P]),
    "mlg_refil_packed_agent_size": (ctypes.c_int64, [_P]),
    "mlg_refil_pack_agent": (ctypes.c_int, [_P, _P, _P, _P]),
    "mlg_refil_agent_forward": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _I, _P]),
    "mlg_refil_rollout": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, ctypes.c_float, _I, _P]),
    "mlg_refil_attention": (ctypes.c_int, [_P] * 6 + [_I] * 4 + [_P] * 7),
    "mlg_refil_packed_mixer_size": (ctypes.c_int64, [_P]),
    "mlg_refil_pack_mixer": (ctypes.c_int, [_P, _P, _P, _P]),
    "mlg_refil_mixer_forward": (ctypes.c_int, [_P] * 7 + [_I, _P, _I, _P]),
    "mlg_refil_param_counts": (ctypes.c_int64, [_P, _P, _P]),
    "mlg_refil_workspace_floats": (ctypes.c_int64, [_P]),
    "mlg_refil_train": (ctypes.c_int, [_P, _P, _P]),
    "mlg_debug_set_stamps": (ctypes.c_int, [_P]),
    "mlg_debug_set_learner_stamps": (ctypes.c_int, [_P]),
    "mlg_refil_debug_set_stamps": (ctypes.c_int, [_P]),
    "mlg_league_record_runs": (ctypes.c_int, [_P, _P, _I, _P, _I, _P]),
    "mlg_refil_draw_groups": (ctypes.c_int, [_I, _I, ctypes.c_uint64, ctypes.c_uint32, _P, _P]),
    "mlg_last_error": (ctypes.c_char_p, []),
    "mlg_version": (ctypes.c_char_p, []),
}

_lib = None


def lib_path() -> str:
    return _LIB_PATH


def load(require_gpu: bool = False):
    """Load libmaleague.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            raise NativeError(f"libmaleague.so not found at {_LIB_PATH}; build it with `make -C ma-league_amd` "
                              "(or __graft_entry__.build()). There is no CPU fallback.")
        lib = ctypes.CDLL(_LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    if require_gpu and not torch.cuda.is_available():
        raise NativeError("maleague kernels need a ROCm GPU (gfx950); torch.cuda.is_available() is False")
    return _lib


def call(name: str, *args) -> None:
    """Invoke a status-returning entry point; raise NativeError with mlg_last_error() on failure."""
    lib = load(require_gpu=True)
    rc = getattr(lib, name)(*args)
    if rc != 0:
        raise NativeError(f"{name} failed: {lib.mlg_last_error().decode()}")


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t: torch.Tensor | None) -> int | None:
    if t is None:
        return None
    if not t.is_cuda:
        raise NativeError(f"maleague kernels need device tensors, got a {t.device} tensor")
    if not t.is_contiguous():
        raise NativeError("maleague kernels need contiguous tensors")
    return t.data_ptr()


def byref(s):
    return ctypes.byref(s)
