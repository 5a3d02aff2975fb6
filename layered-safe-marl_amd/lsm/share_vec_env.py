"""``ShareVecEnv`` -- the reference's abstract vec-env base (``onpolicy/envs/env_wrappers.py:29-140``),
restated so ``GpuGraphVecEnv`` is one by construction.

The runner only uses the attributes set here and ``reset`` / ``step_async`` / ``step_wait`` /
``step`` / ``close``. Inside the reference's process a maintainer registers the GPU env with the
reference's own ABC as well (``onpolicy.envs.env_wrappers.ShareVecEnv.register(GpuGraphVecEnv)``,
INTEGRATION.md), so ``isinstance(envs, ShareVecEnv)`` holds there too.
"""
from __future__ import annotations

from abc import ABC, abstractmethod


class ShareVecEnv(ABC):
    """An abstract asynchronous, vectorized environment (env_wrappers.py:29-140)."""
    closed = False
    viewer = None
    metadata = {"render.modes": ["human", "rgb_array"]}

    # num_envs, observation_space, share_observation_space, action_space are set by the subclass
    # (the reference's __init__ takes them as arguments, env_wrappers.py:42-46)

    @abstractmethod
    def reset(self, num_current_episode: int = 0):
        """Reset all envs; returns the observations (env_wrappers.py:48-58)."""

    @abstractmethod
    def step_async(self, actions, num_current_episode=None):
        """Start a step with the given actions (env_wrappers.py:60-69)."""

    @abstractmethod
    def step_wait(self):
        """Wait for the step started by step_async (env_wrappers.py:71-82)."""

    def close_extras(self):
        """Clean up extra resources beyond the base class (env_wrappers.py:84-89)."""

    def close(self):
        if self.closed:
            return
        self.close_extras()
        self.closed = True

    def step(self, actions, num_current_episode=None):
        """Step synchronously (env_wrappers.py:103-110)."""
        self.step_async(actions, num_current_episode)
        return self.step_wait()

    def render(self, mode="human"):
        raise NotImplementedError("rendering is not on the accelerated path (SURVEY.md section 8)")

    def get_images(self):
        raise NotImplementedError

    @property
    def unwrapped(self):
        return self
