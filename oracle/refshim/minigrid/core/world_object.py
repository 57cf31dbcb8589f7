"""minigrid.core.world_object restatement.

TEST INFRASTRUCTURE ONLY (see package docstring).  Behaviour per type:
can_overlap / can_pickup / see_behind / encode / toggle.
"""
from .constants import COLOR_TO_IDX, OBJECT_TO_IDX


class WorldObj:
    def __init__(self, type, color):
        self.type = type
        self.color = color
        self.contains = None
        self.init_pos = None
        self.cur_pos = None

    def can_overlap(self):
        return False

    def can_pickup(self):
        return False

    def can_contain(self):
        return False

    def see_behind(self):
        return True

    def toggle(self, env, pos):
        return False

    def encode(self):
        return (OBJECT_TO_IDX[self.type], COLOR_TO_IDX[self.color], 0)


class Goal(WorldObj):
    def __init__(self):
        super().__init__("goal", "green")

    def can_overlap(self):
        return True


class Floor(WorldObj):
    def __init__(self, color="blue"):
        super().__init__("floor", color)

    def can_overlap(self):
        return True


class Lava(WorldObj):
    def __init__(self):
        super().__init__("lava", "red")

    def can_overlap(self):
        return True


class Wall(WorldObj):
    def __init__(self, color="grey"):
        super().__init__("wall", color)

    def see_behind(self):
        return False


class Door(WorldObj):
    def __init__(self, color, is_open=False, is_locked=False):
        super().__init__("door", color)
        self.is_open = is_open
        self.is_locked = is_locked

    def can_overlap(self):
        return self.is_open

    def see_behind(self):
        return self.is_open

    def toggle(self, env, pos):
        if self.is_locked:
            if isinstance(env.carrying, Key) and env.carrying.color == self.color:
                self.is_locked = False
                self.is_open = True
                return True
            return False
        self.is_open = not self.is_open
        return True

    def encode(self):
        if self.is_open:
            state = 0
        elif self.is_locked:
            state = 2
        else:
            state = 1
        return (OBJECT_TO_IDX[self.type], COLOR_TO_IDX[self.color], state)


class Key(WorldObj):
    def __init__(self, color="blue"):
        super().__init__("key", color)

    def can_pickup(self):
        return True


class Ball(WorldObj):
    def __init__(self, color="blue"):
        super().__init__("ball", color)

    def can_pickup(self):
        return True


class Box(WorldObj):
    def __init__(self, color, contains=None):
        super().__init__("box", color)
        self.contains = contains

    def can_pickup(self):
        return True

    def can_contain(self):
        return True

    def toggle(self, env, pos):
        env.grid.set(pos[0], pos[1], self.contains)
        return True
