"""QMIX/VDN Q-learner (API of src/marl/learners/learner.py:6-79 and q_learner.py:15-147).

train() is one call into the fused gfx950 pipeline (mlg_qlearner_train): online + target BPTT unrolls,
double-Q targets, mixer forward/backward, masked TD loss, all weight gradients, clip_grad_norm_ and the
RMSprop step. To make that possible the parameters of the MAC and mixer (and of their target copies)
are re-homed into flat fp32 buffers; the nn.Module parameters become views into them, so state_dict()
keys, checkpoint files and torch.optim.RMSprop.state_dict() stay compatible with the reference.
"""
from __future__ import annotations

import copy

import torch

from .. import _native
from ..components.batch_view import mlg_batch
from ..modules.mixers import QMixer, VDNMixer
from ..utils.checkpoint import save_module, save_optimizer

AGENT_ORDER = ["fc1.weight", "fc1.bias", "gru.weight_ih", "gru.weight_hh", "gru.bias_ih", "gru.bias_hh",
               "fc2.weight", "fc2.bias"]
QMIX_ORDER = ["hyper_w_1.0.weight", "hyper_w_1.0.bias", "hyper_w_1.2.weight", "hyper_w_1.2.bias",
              "hyper_w_final.0.weight", "hyper_w_final.0.bias", "hyper_w_final.2.weight", "hyper_w_final.2.bias",
              "hyper_b_1.weight", "hyper_b_1.bias", "V.0.weight", "V.0.bias", "V.2.weight", "V.2.bias"]


class FlatParams:
    """Moves `params` into one contiguous fp32 device buffer; each Parameter becomes a view of it."""

    def __init__(self, params, device):
        params = list(params)
        n = sum(p.numel() for p in params)
        self.flat = torch.empty(n, dtype=torch.float32, device=device)
        self.views = []
        off = 0
        for p in params:
            k = p.numel()
            self.flat[off:off + k].copy_(p.detach().reshape(-1))
            p.data = self.flat[off:off + k].view_as(p)
            self.views.append((p, off, k))
            off += k

    def attach_grads(self, gflat):
        for p, off, k in self.views:
            p.grad = gflat[off:off + k].view_as(p)


class Learner:
    def __init__(self, mac, scheme, logger, args, name=None):
        self.mac = mac
        self.scheme = scheme
        self.logger = logger
        self.args = args
        self.name = f'{"" if name is None else name}_{self.__class__.__name__.lower()}_'
        self.log_stats_t = -self.args.learner_log_interval - 1
        self.optimiser = None

    def parameters(self):
        raise NotImplementedError()

    def train(self, batch, t_env: int, episode_num: int):
        raise NotImplementedError()

    def update_targets(self):
        pass


class QLearner(Learner):
    def __init__(self, mac, scheme, logger, args, name=None):
        super().__init__(mac, scheme, logger, args, name)
        self.last_target_update_episode = 0
        self.mixer = None
        if args.mixer is not None:
            if args.mixer == "vdn":
                self.mixer = VDNMixer()
            elif args.mixer == "qmix":
                self.mixer = QMixer(args)
            else:
                raise ValueError(f"Mixer {args.mixer} not recognised.")
            self.target_mixer = copy.deepcopy(self.mixer)
        self.target_mac = copy.deepcopy(mac)
        self.device = torch.device(getattr(args, "device", "cuda"))
        self._ws = None
        self._stats = None
        self._last_stats = None
        self._stats_fresh = False
        self.train_calls = 0

    def parameters(self):
        # the reference's precedence slip (q_learner.py:30-32) returns [] for IQL; VDN/QMIX are unaffected
        return list(self.mac.parameters()) + (list(self.mixer.parameters()) if self.mixer is not None else [])

    def _target_parameters(self):
        return list(self.target_mac.parameters()) + (list(self.target_mixer.parameters())
                                                     if self.mixer is not None else [])

    def _check_order(self):
        names = [n for n, _ in self.mac.agent.named_parameters()]
        if names != AGENT_ORDER:
            raise RuntimeError(f"agent parameter order {names} != kernel layout {AGENT_ORDER}")
        if isinstance(self.mixer, QMixer):
            names = [n for n, _ in self.mixer.named_parameters()]
            if names != QMIX_ORDER:
                raise RuntimeError(f"mixer parameter order {names} != kernel layout {QMIX_ORDER}")

    def build_optimizer(self):
        self._check_order()
        for m in [self.mac.agent, self.target_mac.agent] + ([self.mixer, self.target_mixer] if self.mixer else []):
            m.to(self.device)
        params = self.parameters()
        self._flat = FlatParams(params, self.device)
        self._tflat = FlatParams(self._target_parameters(), self.device)
        self._grads = torch.zeros_like(self._flat.flat)
        self._sq = torch.zeros_like(self._flat.flat)
        self._flat.attach_grads(self._grads)
        a = self.args
        self.optimiser = torch.optim.RMSprop(params=params, lr=a.lr, alpha=a.optim_alpha, eps=a.optim_eps)
        self._step = torch.zeros((), dtype=torch.float32)
        for p, off, k in self._flat.views:
            self.optimiser.state[p] = {"step": self._step, "square_avg": self._sq[off:off + k].view_as(p)}
        self._stats = torch.zeros(8, dtype=torch.float32, device=self.device)
        self.mac.agent.mark_dirty()
        self.target_mac.agent.mark_dirty()

    def _cfg(self, B, T):
        a = self.args
        d = self.mac.agent.dims()
        mixer = 2 if isinstance(self.mixer, QMixer) else (1 if isinstance(self.mixer, VDNMixer) else 0)
        return _native.MlgLearnerCfg(B=B, T=T, N=a.n_agents, A=a.n_actions, d_obs=d.d_obs, H=a.rnn_hidden_dim,
                             S=int(a.state_shape), E=int(getattr(a, "mixing_embed_dim", 32)),
                             HE=int(getattr(a, "hypernet_embed", 64)), hypernet_layers=int(getattr(a, "hypernet_layers", 1)),
                             mixer=mixer, double_q=int(bool(a.double_q)), obs_last_action=int(bool(a.obs_last_action)),
                             obs_agent_id=int(bool(a.obs_agent_id)), gamma=float(a.gamma), lr=float(a.lr),
                             optim_alpha=float(a.optim_alpha), optim_eps=float(a.optim_eps),
                             grad_norm_clip=float(a.grad_norm_clip))

    def train(self, batch, t_env, episode_num: int):
        """q_learner.py:34-131. `t_env` may also be a zero-argument callable, resolved after the device work
        is queued (lets the caller avoid a host sync before the launch)."""
        if self.optimiser is None:
            raise RuntimeError("call build_optimizer() before train()")
        lib = _native.load(require_gpu=True)
        cfg = self._cfg(batch.batch_size, batch.max_seq_length)
        need = lib.mlg_qlearner_workspace_floats(_native.byref(cfg))
        if need < 0:
            raise _native.NativeError(lib.mlg_last_error().decode())
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.zeros(int(need * 1.25) + 1024, dtype=torch.float32, device=self.device)
        # a sampled view of the device buffer hands its slot map over as a kernel argument (no H2D copy)
        host_rows = getattr(batch, "host_rows", None)
        if host_rows is not None and (batch.batch_size > lib.mlg_qlearner_inline_rows()
                                      or getattr(batch, "_data", None) is not None):
            host_rows = None
        mb, keep = mlg_batch(batch, device_rows=host_rows is None)
        # the target update due after this step (q_learner.py:127-128) is written by the optimizer launch itself
        sync = (episode_num - self.last_target_update_episode) / self.args.target_update_interval >= 1.0
        # no host sync per train step: trained steps accumulate on the device (Agent.trained_steps)
        counter = self.mac.agent.trained_counter(self.device)
        bufs = _native.MlgLearnerBufs(mb, self._flat.flat.data_ptr(), self._grads.data_ptr(), self._sq.data_ptr(),
                                      self._tflat.flat.data_ptr(), self._ws.data_ptr(), self._stats.data_ptr(),
                                      self._tflat.flat.data_ptr() if sync else None, counter.data_ptr(),
                                      None if host_rows is None else host_rows.ctypes.data)
        _native.call("mlg_qlearner_train", _native.byref(cfg), _native.byref(bufs), _native.stream_ptr(self.device))
        del keep
        self._step += 1
        self.mac.agent.mark_dirty()
        self.train_calls += 1
        if sync:
            self.target_mac.agent.mark_dirty()
            self.logger.info(f"Updated {self.name}target network.")
            self.last_target_update_episode = episode_num
        self._stats_fresh = True
        if callable(t_env):  # lazily resolved t_env: the kernels above are already queued
            up = getattr(t_env, "upper", None)
            if up is not None and up() - self.log_stats_t < self.args.learner_log_interval:
                return  # no log due for any t_env still possible: no wait for the runs in flight
            t_env = t_env()
        if t_env - self.log_stats_t >= self.args.learner_log_interval:
            for k, v in self.last_stats.items():
                self.logger.log_stat(self.name + k, v, t_env)
            self.log_stats_t = t_env

    @property
    def last_stats(self):
        """Stats of the latest train() (q_learner.py:115-124 values); reading them syncs the stream."""
        if self._stats is None or not self._stats_fresh:
            return self._last_stats
        st = self._stats.cpu()
        self._last_stats = {"loss": float(st[0]), "grad_norm": float(st[1]), "td_error_abs": float(st[2]),
                            "q_taken_mean": float(st[3]), "target_mean": float(st[4])}
        self._stats_fresh = False
        return self._last_stats

    def update_targets(self):
        self._tflat.flat.copy_(self._flat.flat)
        self.target_mac.agent.mark_dirty()
        self.logger.info(f"Updated {self.name}target network.")

    def cuda(self):
        pass

    def save_models(self, path, name):
        self.mac.save_models(path, name=self.name)
        if self.mixer is not None:
            save_module(self.mixer, f"{path}/{self.name}mixer.th")
        save_optimizer(self.optimiser, f"{path}/{self.name}opt.th")

    def load_models(self, path):
        self.mac.load_models(path, self.name)
        self.target_mac.load_models(path, self.name)  # target nets are not saved (q_learner.py:141-142)
        if self.mixer is not None:
            sd = torch.load(f"{path}/{self.name}mixer.th", map_location=lambda s, loc: s, weights_only=True)
            self.mixer.load_state_dict(sd)
        opt = torch.load(f"{path}/{self.name}opt.th", map_location=lambda s, loc: s, weights_only=True)
        self.optimiser.load_state_dict(opt)
        for p, off, k in self._flat.views:  # re-home the loaded RMSprop state into the flat buffer
            st = self.optimiser.state.get(p, {})
            if "square_avg" in st:
                self._sq[off:off + k].copy_(st["square_avg"].reshape(-1))
            if "step" in st:  # one shared step counter (RMSprop steps every parameter together)
                self._step.fill_(float(st["step"]))
            self.optimiser.state[p] = {"step": self._step, "square_avg": self._sq[off:off + k].view_as(p)}
        self.mac.agent.mark_dirty()
        self.target_mac.agent.mark_dirty()
