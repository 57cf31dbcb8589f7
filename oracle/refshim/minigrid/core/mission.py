"""minigrid.core.mission restatement: only the constructor is exercised."""


class MissionSpace:
    def __init__(self, mission_func, ordered_placeholders=None, max_length=200):
        self.mission_func = mission_func
        self.ordered_placeholders = ordered_placeholders
        self.max_length = max_length
