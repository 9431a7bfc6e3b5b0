"""Action spaces of the reference (``Action_Spaces/``)."""
import numpy as np


class Base_Space(object):
    """``Action_Spaces/base_space.py:3-12``."""

    def sample(self):
        raise NotImplementedError()


class Discrete(Base_Space):
    """``Action_Spaces/discrete.py:4-14``: ``sample(s)`` = randint(num_actions)."""

    def __init__(self, num_actions):
        self.num_actions = num_actions

    def sample(self, s=None):
        return np.random.randint(self.num_actions, size=s)


class Continuous(Base_Space):
    """``Action_Spaces/continuous.py:4-16``."""

    def __init__(self, low, high):
        self.low = low
        self.high = high
        self.interval = np.array([low, high])

    def sample(self, s=None):
        return np.random.uniform(self.low, self.high, size=s)
