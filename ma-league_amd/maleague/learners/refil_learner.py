"""REFILLearner (API of src/marl/learners/refil_learner.py:46-267) on the fused gfx950 pipeline.

train() is one call into mlg_refil_train: the EntityMAC unrolls of the plain, within-group and interact-group
copies (the imagine agent, entity_rnn_agent.py:88-126) and of the target MAC, FlexQMixer on the plain and the
imagined chosen Q, double-Q targets through the target mixer, the lambda-mixed TD loss, every gradient,
clip_grad_norm_ and RMSprop. As in QLearner the nn.Module parameters are views into flat fp32 buffers, so
state_dict() keys and the .th checkpoint files stay those of the reference.
"""
from __future__ import annotations

import copy

import torch

from .. import _native
from ..components.batch_view import mlg_entity_batch
from ..modules.mixers import FlexQMixer
from ..utils.checkpoint import save_module, save_optimizer
from .q_learner import FlatParams, Learner

AGENT_ORDER = ["fc1.weight", "fc1.bias", "attn.in_trans.weight", "attn.out_trans.weight", "attn.out_trans.bias",
               "fc2.weight", "fc2.bias", "rnn.weight_ih", "rnn.weight_hh", "rnn.bias_ih", "rnn.bias_hh", "fc3.weight",
               "fc3.bias"]
HYPER_ORDER = ["fc1.weight", "fc1.bias", "attn.in_trans.weight", "attn.out_trans.weight", "attn.out_trans.bias",
               "fc2.weight", "fc2.bias"]
MIXER_ORDER = [f"{h}.{p}" for h in ("hyper_w_1", "hyper_w_final", "hyper_b_1", "V") for p in HYPER_ORDER]


class REFILLearner(Learner):
    def __init__(self, mac, scheme, logger, args, name=None):
        super().__init__(mac, scheme, logger, args, name)
        if args.mixer != "flex_qmix":
            raise ValueError(f"REFILLearner: mixer {args.mixer!r} not built (flex_qmix is the REFIL mixer)")
        if "imagine" not in args.agent:
            raise NotImplementedError("REFILLearner: the imagine agent is the built path (refil_learner.py:122)")
        if getattr(args, "weight_decay", 0):
            raise NotImplementedError("RMSprop weight_decay != 0 is not built")
        self.last_target_update_episode = 0
        self.mixer = FlexQMixer(args)
        self.target_mixer = copy.deepcopy(self.mixer)
        self.target_mac = copy.deepcopy(mac)
        self.device = torch.device(getattr(args, "device", "cuda"))
        self._ws = None
        self._stats = None
        self._last_stats = None
        self._stats_fresh = False
        self.train_calls = 0
        self._groups = None  # device buffer of the imagine group draw
        self._group_seed = (int(getattr(args, "seed", 0)) << 32) ^ 0x5EF11  # key of the draw's counter-based RNG

    def parameters(self):
        return list(self.mac.parameters()) + list(self.mixer.parameters())

    def _target_parameters(self):
        return list(self.target_mac.parameters()) + list(self.target_mixer.parameters())

    def _check_order(self):
        names = [n for n, _ in self.mac.agent.named_parameters()]
        if names != AGENT_ORDER:
            raise RuntimeError(f"agent parameter order {names} != kernel layout {AGENT_ORDER}")
        names = [n for n, _ in self.mixer.named_parameters()]
        if names != MIXER_ORDER:
            raise RuntimeError(f"mixer parameter order {names} != kernel layout {MIXER_ORDER}")

    def build_optimizer(self):
        self._check_order()
        for m in (self.mac.agent, self.target_mac.agent, self.mixer, self.target_mixer):
            m.to(self.device)
        params = self.parameters()
        self._flat = FlatParams(params, self.device)
        self._tflat = FlatParams(self._target_parameters(), self.device)
        self._grads = torch.zeros_like(self._flat.flat)
        self._sq = torch.zeros_like(self._flat.flat)
        self._flat.attach_grads(self._grads)
        a = self.args
        self.optimiser = torch.optim.RMSprop(params=params, lr=a.lr, alpha=a.optim_alpha, eps=a.optim_eps,
                                             weight_decay=getattr(a, "weight_decay", 0))
        self._step = torch.zeros((), dtype=torch.float32)
        for p, off, k in self._flat.views:
            self.optimiser.state[p] = {"step": self._step, "square_avg": self._sq[off:off + k].view_as(p)}
        self._stats = torch.zeros(8, dtype=torch.float32, device=self.device)
        self.mac.agent.mark_dirty()
        self.target_mac.agent.mark_dirty()

    def _cfg(self, B, T):
        a = self.args
        d = self.mac.agent.dims()
        return _native.MlgRefilLearnerCfg(
            B=B, T=T, n_agents=a.n_agents, n_entities=a.n_entities, entity_shape=d.entity_shape, n_actions=a.n_actions,
            entity_last_action=d.entity_last_action, attn_embed_dim=a.attn_embed_dim, attn_n_heads=a.attn_n_heads,
            rnn_hidden_dim=a.rnn_hidden_dim, hypernet_embed=a.hypernet_embed, mixing_embed_dim=a.mixing_embed_dim,
            double_q=int(bool(a.double_q)), softmax_mixing_weights=int(bool(a.softmax_mixing_weights)), imagine=1,
            gamma=float(a.gamma), lmbda=float(a.lmbda), lr=float(a.lr), optim_alpha=float(a.optim_alpha),
            optim_eps=float(a.optim_eps), grad_norm_clip=float(a.grad_norm_clip))

    def train(self, batch, t_env, episode_num: int, groupA=None):
        """refil_learner.py:102-237. groupA [B, NE] (or [B, 1, NE]) uint8: the imagine group draw; drawn on the
        device when None (the reference's th.rand + th.bernoulli, entity_rnn_agent.py:95-97)."""
        if self.optimiser is None:
            raise RuntimeError("call build_optimizer() before train()")
        lib = _native.load(require_gpu=True)
        B, NE = batch.batch_size, self.args.n_entities
        cfg = self._cfg(B, batch.max_seq_length)
        need = lib.mlg_refil_workspace_floats(_native.byref(cfg))
        if need < 0:
            raise _native.NativeError(lib.mlg_last_error().decode())
        if self._ws is None or self._ws.numel() < need:
            self._ws = None
            self._ws = torch.zeros(int(need * 1.1) + 1024, dtype=torch.float32, device=self.device)
        if groupA is None:  # drawn on the device: one launch (mlg_refil_draw_groups), counter = train call
            if self._groups is None or self._groups.shape != (B, NE):
                self._groups = torch.empty(B, NE, dtype=torch.uint8, device=self.device)
            groupA = self._groups
            _native.call("mlg_refil_draw_groups", B, NE, self._group_seed, self.train_calls & 0xFFFFFFFF,
                         groupA.data_ptr(), _native.stream_ptr(self.device))
        groupA = groupA.reshape(B, NE).to(device=self.device, dtype=torch.uint8).contiguous()
        # a sampled view's slot map travels as a kernel argument (no pinned host copy + H2D copy per call)
        host_rows = getattr(batch, "host_rows", None)
        if host_rows is not None and (B > lib.mlg_qlearner_inline_rows() or getattr(batch, "_data", None) is not None):
            host_rows = None
        mb, keep = mlg_entity_batch(batch, device_rows=host_rows is None)
        # trained steps accumulate on the device inside the optimizer launch (no separate add); the target update
        # due after this step (refil_learner.py:181-183) is written by that launch too (no separate copy)
        counter = self.mac.agent.trained_counter(self.device)
        sync = (episode_num - self.last_target_update_episode) / self.args.target_update_interval >= 1.0
        bufs = _native.MlgRefilLearnerBufs(mb, groupA.data_ptr(), self._flat.flat.data_ptr(), self._grads.data_ptr(),
                                           self._sq.data_ptr(), self._tflat.flat.data_ptr(), self._ws.data_ptr(),
                                           self._stats.data_ptr(), counter.data_ptr(),
                                           self._tflat.flat.data_ptr() if sync else None,
                                           None if host_rows is None else host_rows.ctypes.data)
        _native.call("mlg_refil_train", _native.byref(cfg), _native.byref(bufs), _native.stream_ptr(self.device))
        del keep
        self._groupA = groupA
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
            # the reference REFIL learner logs unprefixed keys, im_loss only for imagine agents
            # (refil_learner.py:185-195; unlike QLearner's "{name}loss" keys)
            imagine = "imagine" in str(getattr(self.args, "agent", ""))
            for k, v in self.last_stats.items():
                if k == "im_loss" and not imagine:
                    continue
                self.logger.log_stat(k, v, t_env)
            self.log_stats_t = t_env

    @property
    def last_stats(self):
        """Stats of the latest train() (refil_learner.py:220-231 keys); reading them syncs the stream."""
        if self._stats is None or not self._stats_fresh:
            return self._last_stats
        st = self._stats.cpu()
        self._last_stats = {"loss": float(st[0]), "im_loss": float(st[1]), "grad_norm": float(st[2]),
                            "td_error_abs": float(st[3]), "q_taken_mean": float(st[4]), "target_mean": float(st[5])}
        self._stats_fresh = False
        return self._last_stats

    def update_targets(self):
        self._tflat.flat.copy_(self._flat.flat)
        self.target_mac.agent.mark_dirty()
        self.logger.info(f"Updated {self.name}target network.")

    def cuda(self):
        pass

    def save_models(self, path, name=None):
        name = self.name if name is None else name
        self.mac.save_models(path, name=name)
        save_module(self.mixer, f"{path}/{name}mixer.th")
        save_optimizer(self.optimiser, f"{path}/{name}opt.th")

    def load_models(self, path):
        self.mac.load_models(path, self.name)
        self.target_mac.load_models(path, self.name)
        self.mixer.load_state_dict(torch.load(f"{path}/{self.name}mixer.th", map_location=lambda s, loc: s,
                                              weights_only=True))
        self.target_mixer.load_state_dict(self.mixer.state_dict())
        opt = torch.load(f"{path}/{self.name}opt.th", map_location=lambda s, loc: s, weights_only=True)
        self.optimiser.load_state_dict(opt)
        for p, off, k in self._flat.views:
            st = self.optimiser.state.get(p, {})
            if "square_avg" in st:
                self._sq[off:off + k].copy_(st["square_avg"].reshape(-1))
            if "step" in st:
                self._step.fill_(float(st["step"]))
            self.optimiser.state[p] = {"step": self._step, "square_avg": self._sq[off:off + k].view_as(p)}
        self.mac.agent.mark_dirty()
        self.target_mac.agent.mark_dirty()
