"""minigrid.core.grid restatement.

TEST INFRASTRUCTURE ONLY.  Storage is row-major `j*W+i`; `slice` pads out of
bounds with Wall(); `rotate_left` maps old (i,j) -> new (j, H-1-i).
"""
import numpy as np

from .constants import OBJECT_TO_IDX
from .world_object import Wall


class Grid:
    def __init__(self, width, height):
        assert width >= 3 and height >= 3
        self.width = width
        self.height = height
        self.grid = [None] * (width * height)

    def set(self, i, j, v):
        assert 0 <= i < self.width, f"column index {i} outside of grid of width {self.width}"
        assert 0 <= j < self.height, f"row index {j} outside of grid of height {self.height}"
        self.grid[j * self.width + i] = v

    def get(self, i, j):
        assert 0 <= i < self.width
        assert 0 <= j < self.height
        return self.grid[j * self.width + i]

    def horz_wall(self, x, y, length=None, obj_type=Wall):
        if length is None:
            length = self.width - x
        for i in range(0, length):
            self.set(x + i, y, obj_type())

    def vert_wall(self, x, y, length=None, obj_type=Wall):
        if length is None:
            length = self.height - y
        for j in range(0, length):
            self.set(x, y + j, obj_type())

    def wall_rect(self, x, y, w, h):
        self.horz_wall(x, y, w)
        self.horz_wall(x, y + h - 1, w)
        self.vert_wall(x, y, h)
        self.vert_wall(x + w - 1, y, h)

    def rotate_left(self):
        grid = Grid(self.height, self.width)
        for i in range(self.width):
            for j in range(self.height):
                v = self.get(i, j)
                grid.set(j, grid.height - 1 - i, v)
        return grid

    def slice(self, topX, topY, width, height):
        grid = Grid(width, height)
        for j in range(0, height):
            for i in range(0, width):
                x = topX + i
                y = topY + j
                if 0 <= x < self.width and 0 <= y < self.height:
                    v = self.get(x, y)
                else:
                    v = Wall()
                grid.set(i, j, v)
        return grid

    def encode(self, vis_mask=None):
        if vis_mask is None:
            vis_mask = np.ones((self.width, self.height), dtype=bool)
        array = np.zeros((self.width, self.height, 3), dtype="uint8")
        for i in range(self.width):
            for j in range(self.height):
                if vis_mask[i, j]:
                    v = self.get(i, j)
                    if v is None:
                        array[i, j, 0] = OBJECT_TO_IDX["empty"]
                        array[i, j, 1] = 0
                        array[i, j, 2] = 0
                    else:
                        array[i, j, :] = v.encode()
        return array

    def process_vis(self, agent_pos):
        mask = np.zeros(shape=(self.width, self.height), dtype=bool)
        mask[agent_pos[0], agent_pos[1]] = True
        for j in reversed(range(0, self.height)):
            for i in range(0, self.width - 1):
                if not mask[i, j]:
                    continue
                cell = self.get(i, j)
                if cell and not cell.see_behind():
                    continue
                mask[i + 1, j] = True
                if j > 0:
                    mask[i + 1, j - 1] = True
                    mask[i, j - 1] = True
            for i in reversed(range(1, self.width)):
                if not mask[i, j]:
                    continue
                cell = self.get(i, j)
                if cell and not cell.see_behind():
                    continue
                mask[i - 1, j] = True
                if j > 0:
                    mask[i - 1, j - 1] = True
                    mask[i, j - 1] = True
        for j in range(0, self.height):
            for i in range(0, self.width):
                if not mask[i, j]:
                    self.set(i, j, None)
        return mask
