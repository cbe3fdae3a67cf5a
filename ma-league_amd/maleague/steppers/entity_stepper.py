"""ParallelStepper over the entity env (REFIL, config 5).

Same run semantics, async run summary and zero-copy replay insert as ParallelStepper
(src/steppers/parallel_stepper.py:82-216); the batch follows the entity scheme (entities, obs_mask,
entity_mask, avail_actions, actions, reward, terminated) and the MAC is an EntityMAC, fused into one launch of
mlg_refil_rollout per run.
"""
from __future__ import annotations

from .. import _native
from ..components.batch_view import mlg_entity_batch
from ..envs.entity_env import EntityEnvSpec
from .parallel_stepper import EpisodeStepper, ParallelStepper


class EntityParallelStepper(ParallelStepper):
    _batch_keys = ("entities", "obs_mask", "entity_mask", "actions", "avail_actions", "reward", "terminated",
                   "actions_onehot", "filled")

    def _build_spec(self, env_args, config_dir):
        return EntityEnvSpec.from_env_args(env_args, config_dir)

    def _to_mlg(self, batch):
        return mlg_entity_batch(batch)

    def _rollout(self, mb, run_info, epsilon, test_mode):
        agent = self.home_mac.agent
        st = self.envs.to_c()
        _native.call("mlg_refil_rollout", _native.byref(self._cspec), _native.byref(st), _native.byref(agent.dims()),
                     _native.ptr(agent.packed()), _native.byref(mb), _native.byref(run_info), float(epsilon),
                     int(bool(test_mode)), _native.stream_ptr(self.device))


class EntityEpisodeStepper(EntityParallelStepper, EpisodeStepper):
    """B = 1 variant (episode_stepper.py:16-186 over the entity env)."""
