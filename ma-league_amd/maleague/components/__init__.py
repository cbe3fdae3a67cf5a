from .episode_batch import EpisodeBatch
from .replay_buffer import ReplayBuffer
from .transforms import OneHot, Transform
from .epsilon_schedules import DecayThenFlatSchedule

__all__ = ["EpisodeBatch", "ReplayBuffer", "OneHot", "Transform", "DecayThenFlatSchedule"]
