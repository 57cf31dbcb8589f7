"""minigrid.core.actions restatement (`custom_env.py:41-51`)."""
from enum import IntEnum


class Actions(IntEnum):
    left = 0
    right = 1
    forward = 2
    pickup = 3
    drop = 4
    toggle = 5
    done = 6
