"""Terrain heightfield generator (humanoid/utils/terrain.py:38-231 of the reference).

``Terrain`` lays out ``num_rows x num_cols`` sub-terrains of ``terrain_length x terrain_width`` m
at ``horizontal_scale`` m per pixel with a ``border_size`` m flat border, into one int16
heightfield (units of ``vertical_scale`` m).  Row index = world x + border, column = world y +
border (the heightfield transform of humanoid_env.py:363-380).  ``env_origins[i, j]`` is the
centre of sub-terrain (i, j) at the maximum height of its central 2 x 2 m.

``HumanoidTerrain`` is the XBot profile: a random (type, difficulty) per sub-terrain drawn from
numpy's global RNG, with the mix of ``terrain_proportions`` (flat, obstacles, random uniform,
slope up, slope down, stairs up, stairs down).  The device copy of ``heightsamples`` is what
K_step collides against (csrc/hg_physics2.hip ``ground``) and what the measured-heights path
samples.  Primitive functions: humanoid/utils/terrain_utils.py (parity unpinned, see there).
"""
import numpy as np

from . import terrain_utils


class Terrain:
    def __init__(self, cfg, num_robots) -> None:
        self.cfg = cfg
        self.num_robots = num_robots
        self.type = cfg.mesh_type
        if self.type in ["none", "plane"]:
            return
        self.env_length = cfg.terrain_length
        self.env_width = cfg.terrain_width
        self.proportions = list(np.cumsum(cfg.terrain_proportions))
        self.cfg.num_sub_terrains = cfg.num_rows * cfg.num_cols
        self.env_origins = np.zeros((cfg.num_rows, cfg.num_cols, 3))
        self.width_per_env_pixels = int(self.env_width / cfg.horizontal_scale)
        self.length_per_env_pixels = int(self.env_length / cfg.horizontal_scale)
        self.border = int(cfg.border_size / cfg.horizontal_scale)
        self.tot_cols = int(cfg.num_cols * self.width_per_env_pixels) + 2 * self.border
        self.tot_rows = int(cfg.num_rows * self.length_per_env_pixels) + 2 * self.border
        self.height_field_raw = np.zeros((self.tot_rows, self.tot_cols), dtype=np.int16)
        if cfg.curriculum:
            self.curiculum()
        elif cfg.selected:
            self.selected_terrain()
        else:
            self.randomized_terrain()
        self.heightsamples = self.height_field_raw
        if self.type == "trimesh":
            self.vertices, self.triangles = terrain_utils.convert_heightfield_to_trimesh(
                self.height_field_raw, cfg.horizontal_scale, cfg.vertical_scale, cfg.slope_treshold)

    def _sub(self):
        return terrain_utils.SubTerrain("terrain", width=self.width_per_env_pixels, length=self.width_per_env_pixels,
                                        vertical_scale=self.cfg.vertical_scale,
                                        horizontal_scale=self.cfg.horizontal_scale)

    def randomized_terrain(self):
        for k in range(self.cfg.num_sub_terrains):
            i, j = np.unravel_index(k, (self.cfg.num_rows, self.cfg.num_cols))
            choice = np.random.uniform(0, 1)
            difficulty = np.random.choice([0.5, 0.75, 0.9])
            self.add_terrain_to_map(self.make_terrain(choice, difficulty), i, j)

    def curiculum(self):  # (sic) the reference's method name
        for j in range(self.cfg.num_cols):
            for i in range(self.cfg.num_rows):
                difficulty = i / self.cfg.num_rows
                choice = j / self.cfg.num_cols + 0.001
                self.add_terrain_to_map(self.make_terrain(choice, difficulty), i, j)

    def selected_terrain(self):
        """One primitive for every sub-terrain: ``terrain_kwargs = {"type": name, "terrain_kwargs":
        {...}}`` with ``name`` a terrain_utils function (the reference eval()s the name)."""
        kw = dict(self.cfg.terrain_kwargs)
        name = kw.pop("type")
        fn = getattr(terrain_utils, name.split(".")[-1])
        args = kw.get("terrain_kwargs", kw)
        for k in range(self.cfg.num_sub_terrains):
            i, j = np.unravel_index(k, (self.cfg.num_rows, self.cfg.num_cols))
            t = self._sub()
            fn(t, **args)
            self.add_terrain_to_map(t, i, j)

    def make_terrain(self, choice, difficulty):
        t = self._sub()
        p = self.proportions
        slope = difficulty * 0.4
        step_height = 0.05 + 0.18 * difficulty
        discrete_obstacles_height = 0.05 + difficulty * 0.2
        stepping_stones_size = 1.5 * (1.05 - difficulty)
        stone_distance = 0.05 if difficulty == 0 else 0.1
        gap_size = 1.0 * difficulty
        pit_depth = 1.0 * difficulty
        if choice < p[0]:
            if choice < p[0] / 2:
                slope *= -1
            terrain_utils.pyramid_sloped_terrain(t, slope=slope, platform_size=3.0)
        elif choice < p[1]:
            terrain_utils.pyramid_sloped_terrain(t, slope=slope, platform_size=3.0)
            terrain_utils.random_uniform_terrain(t, min_height=-0.05, max_height=0.05, step=0.005,
                                                 downsampled_scale=0.2)
        elif choice < p[3]:
            if choice < p[2]:
                step_height *= -1
            terrain_utils.pyramid_stairs_terrain(t, step_width=0.31, step_height=step_height, platform_size=3.0)
        elif choice < p[4]:
            terrain_utils.discrete_obstacles_terrain(t, discrete_obstacles_height, 1.0, 2.0, 20, platform_size=3.0)
        elif choice < p[5]:
            terrain_utils.stepping_stones_terrain(t, stone_size=stepping_stones_size, stone_distance=stone_distance,
                                                  max_height=0.0, platform_size=4.0)
        elif choice < p[6]:
            gap_terrain(t, gap_size=gap_size, platform_size=3.0)
        else:
            pit_terrain(t, depth=pit_depth, platform_size=4.0)
        return t

    def add_terrain_to_map(self, terrain, row, col):
        lp, wp = self.length_per_env_pixels, self.width_per_env_pixels
        sx, sy = self.border + row * lp, self.border + col * wp
        self.height_field_raw[sx:sx + lp, sy:sy + wp] = terrain.height_field_raw
        hs = terrain.horizontal_scale
        x1, x2 = int((self.env_length / 2.0 - 1) / hs), int((self.env_length / 2.0 + 1) / hs)
        y1, y2 = int((self.env_width / 2.0 - 1) / hs), int((self.env_width / 2.0 + 1) / hs)
        z = np.max(terrain.height_field_raw[x1:x2, y1:y2]) * terrain.vertical_scale
        self.env_origins[row, col] = [(row + 0.5) * self.env_length, (col + 0.5) * self.env_width, z]


def gap_terrain(terrain, gap_size, platform_size=1.0):
    """A square moat of width ``gap_size`` m around a ``platform_size`` m platform."""
    gap = int(gap_size / terrain.horizontal_scale)
    plat = int(platform_size / terrain.horizontal_scale)
    cx, cy = terrain.length // 2, terrain.width // 2
    x1 = (terrain.length - plat) // 2
    y1 = (terrain.width - plat) // 2
    x2, y2 = x1 + gap, y1 + gap
    terrain.height_field_raw[cx - x2:cx + x2, cy - y2:cy + y2] = -1000
    terrain.height_field_raw[cx - x1:cx + x1, cy - y1:cy + y1] = 0


def pit_terrain(terrain, depth, platform_size=1.0):
    """A central square pit ``depth`` m deep."""
    d = int(depth / terrain.vertical_scale)
    half = int(platform_size / terrain.horizontal_scale / 2)
    x1, x2 = terrain.length // 2 - half, terrain.length // 2 + half
    y1, y2 = terrain.width // 2 - half, terrain.width // 2 + half
    terrain.height_field_raw[x1:x2, y1:y2] = -d


class HumanoidTerrain(Terrain):
    """XBot profile (terrain.py:189-231): difficulty ~ U[0,1); obstacles <= 0.04 m, random
    uniform +-0.07 m, slopes <= 0.15, stairs of 0.4 m treads."""

    def randomized_terrain(self):
        for k in range(self.cfg.num_sub_terrains):
            i, j = np.unravel_index(k, (self.cfg.num_rows, self.cfg.num_cols))
            choice = np.random.uniform(0, 1)
            difficulty = np.random.uniform(0, 1)
            self.add_terrain_to_map(self.make_terrain(choice, difficulty), i, j)

    def make_terrain(self, choice, difficulty):
        t = self._sub()
        p = self.proportions
        obstacle_h = difficulty * 0.04
        r_height = difficulty * 0.07
        h_slope = difficulty * 0.15
        if choice < p[0]:
            pass
        elif choice < p[1]:
            terrain_utils.discrete_obstacles_terrain(t, obstacle_h, 1.0, 2.0, 20, platform_size=3.0)
        elif choice < p[2]:
            terrain_utils.random_uniform_terrain(t, min_height=-r_height, max_height=r_height, step=0.005,
                                                 downsampled_scale=0.2)
        elif choice < p[3]:
            terrain_utils.pyramid_sloped_terrain(t, slope=h_slope, platform_size=0.1)
        elif choice < p[4]:
            terrain_utils.pyramid_sloped_terrain(t, slope=-h_slope, platform_size=0.1)
        elif choice < p[5]:
            terrain_utils.pyramid_stairs_terrain(t, step_width=0.4, step_height=obstacle_h, platform_size=1.0)
        elif choice < p[6]:
            terrain_utils.pyramid_stairs_terrain(t, step_width=0.4, step_height=-obstacle_h, platform_size=1.0)
        return t
