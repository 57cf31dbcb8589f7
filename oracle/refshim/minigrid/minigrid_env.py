"""minigrid.minigrid_env.MiniGridEnv restatement.

TEST INFRASTRUCTURE ONLY.  Restates reset / step / gen_obs / place_obj /
place_agent / put_obj / _reward exactly as the public minigrid 2.x/3.x source
defines them.  `max_tries` is honoured so a live-locked generator raises
instead of hanging (the reference itself would hang).
"""
import math

import numpy as np

import gymnasium as gym

from .core.actions import Actions
from .core.constants import DIR_TO_VEC
from .core.grid import Grid


class MiniGridEnv(gym.Env):
    def __init__(self, mission_space, grid_size=None, width=None, height=None,
                 max_steps=100, see_through_walls=False, agent_view_size=7,
                 render_mode=None, screen_size=640, highlight=True, tile_size=32,
                 agent_pov=False):
        if grid_size:
            width = height = grid_size
        self.mission_space = mission_space
        self.actions = Actions
        self.action_space = gym.spaces.Discrete(len(self.actions))
        assert agent_view_size % 2 == 1 and agent_view_size >= 3
        self.agent_view_size = agent_view_size
        image_space = gym.spaces.Box(low=0, high=255,
                                     shape=(agent_view_size, agent_view_size, 3),
                                     dtype="uint8")
        self.observation_space = gym.spaces.Dict({
            "image": image_space,
            "direction": gym.spaces.Discrete(4),
            "mission": gym.spaces.Text(max_length=200),
        })
        self.render_mode = render_mode
        self.width = width
        self.height = height
        self.max_steps = max_steps
        self.see_through_walls = see_through_walls
        self.agent_pos = (-1, -1)
        self.agent_dir = -1
        self.grid = Grid(width, height)
        self.carrying = None
        self.step_count = 0

    # -- episode ---------------------------------------------------------
    def reset(self, *, seed=None, options=None):
        super().reset(seed=seed)
        self.agent_pos = (-1, -1)
        self.agent_dir = -1
        self._gen_grid(self.width, self.height)
        assert (self.agent_pos >= (0, 0) if isinstance(self.agent_pos, tuple)
                else all(self.agent_pos >= 0) and self.agent_dir >= 0)
        start_cell = self.grid.get(*self.agent_pos)
        assert start_cell is None or start_cell.can_overlap()
        self.carrying = None
        self.step_count = 0
        obs = self.gen_obs()
        return obs, {}

    def _reward(self):
        return 1 - 0.9 * (self.step_count / self.max_steps)

    def _rand_int(self, low, high):
        return self.np_random.integers(low, high)

    def put_obj(self, obj, i, j):
        self.grid.set(i, j, obj)
        obj.init_pos = (i, j)
        obj.cur_pos = (i, j)

    def place_obj(self, obj, top=None, size=None, reject_fn=None, max_tries=math.inf):
        if top is None:
            top = (0, 0)
        else:
            top = (max(top[0], 0), max(top[1], 0))
        if size is None:
            size = (self.grid.width, self.grid.height)
        num_tries = 0
        while True:
            if num_tries > max_tries:
                raise RecursionError("rejection sampling failed in place_obj")
            num_tries += 1
            pos = (
                self._rand_int(top[0], min(top[0] + size[0], self.grid.width)),
                self._rand_int(top[1], min(top[1] + size[1], self.grid.height)),
            )
            if self.grid.get(*pos) is not None:
                continue
            if np.array_equal(pos, self.agent_pos):
                continue
            if reject_fn and reject_fn(self, pos):
                continue
            break
        self.grid.set(pos[0], pos[1], obj)
        if obj is not None:
            obj.init_pos = pos
            obj.cur_pos = pos
        return pos

    def place_agent(self, top=None, size=None, rand_dir=True, max_tries=math.inf):
        self.agent_pos = (-1, -1)
        pos = self.place_obj(None, top, size, max_tries=max_tries)
        self.agent_pos = pos
        if rand_dir:
            self.agent_dir = self._rand_int(0, 4)
        return pos

    # -- geometry --------------------------------------------------------
    @property
    def dir_vec(self):
        assert 0 <= self.agent_dir < 4
        return DIR_TO_VEC[self.agent_dir]

    @property
    def right_vec(self):
        dx, dy = self.dir_vec
        return np.array((-dy, dx))

    @property
    def front_pos(self):
        return self.agent_pos + self.dir_vec

    def get_view_exts(self, agent_view_size=None):
        agent_view_size = agent_view_size or self.agent_view_size
        if self.agent_dir == 0:
            topX = self.agent_pos[0]
            topY = self.agent_pos[1] - agent_view_size // 2
        elif self.agent_dir == 1:
            topX = self.agent_pos[0] - agent_view_size // 2
            topY = self.agent_pos[1]
        elif self.agent_dir == 2:
            topX = self.agent_pos[0] - agent_view_size + 1
            topY = self.agent_pos[1] - agent_view_size // 2
        elif self.agent_dir == 3:
            topX = self.agent_pos[0] - agent_view_size // 2
            topY = self.agent_pos[1] - agent_view_size + 1
        else:
            assert False, "invalid agent direction"
        botX = topX + agent_view_size
        botY = topY + agent_view_size
        return topX, topY, botX, botY

    # -- step ------------------------------------------------------------
    def step(self, action):
        self.step_count += 1
        reward = 0
        terminated = False
        truncated = False
        fwd_pos = self.front_pos
        fwd_cell = self.grid.get(*fwd_pos)
        if action == self.actions.left:
            self.agent_dir -= 1
            if self.agent_dir < 0:
                self.agent_dir += 4
        elif action == self.actions.right:
            self.agent_dir = (self.agent_dir + 1) % 4
        elif action == self.actions.forward:
            if fwd_cell is None or fwd_cell.can_overlap():
                self.agent_pos = tuple(fwd_pos)
            if fwd_cell is not None and fwd_cell.type == "goal":
                terminated = True
                reward = self._reward()
            if fwd_cell is not None and fwd_cell.type == "lava":
                terminated = True
        elif action == self.actions.pickup:
            if fwd_cell and fwd_cell.can_pickup():
                if self.carrying is None:
                    self.carrying = fwd_cell
                    self.carrying.cur_pos = np.array([-1, -1])
                    self.grid.set(fwd_pos[0], fwd_pos[1], None)
        elif action == self.actions.drop:
            if not fwd_cell and self.carrying:
                self.grid.set(fwd_pos[0], fwd_pos[1], self.carrying)
                self.carrying.cur_pos = fwd_pos
                self.carrying = None
        elif action == self.actions.toggle:
            if fwd_cell:
                fwd_cell.toggle(self, fwd_pos)
        elif action == self.actions.done:
            pass
        else:
            raise ValueError(f"Unknown action: {action}")
        if self.step_count >= self.max_steps:
            truncated = True
        obs = self.gen_obs()
        return obs, reward, terminated, truncated, {}

    # -- observation -----------------------------------------------------
    def gen_obs_grid(self, agent_view_size=None):
        topX, topY, botX, botY = self.get_view_exts(agent_view_size)
        agent_view_size = agent_view_size or self.agent_view_size
        grid = self.grid.slice(topX, topY, agent_view_size, agent_view_size)
        for i in range(self.agent_dir + 1):
            grid = grid.rotate_left()
        if not self.see_through_walls:
            vis_mask = grid.process_vis(agent_pos=(agent_view_size // 2, agent_view_size - 1))
        else:
            vis_mask = np.ones(shape=(grid.width, grid.height), dtype=bool)
        agent_pos = grid.width // 2, grid.height - 1
        if self.carrying:
            grid.set(*agent_pos, self.carrying)
        else:
            grid.set(*agent_pos, None)
        return grid, vis_mask

    def gen_obs(self):
        grid, vis_mask = self.gen_obs_grid()
        image = grid.encode(vis_mask)
        return {"image": image, "direction": self.agent_dir, "mission": self.mission}
