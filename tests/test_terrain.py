"""Terrain generator (humanoid/utils/terrain.py, restating the reference's utils/terrain.py and the
isaacgym terrain_utils primitives — parity unpinned, so these are property tests)."""
import numpy as np

from humanoid.envs import XBotLCfg
from humanoid.utils import terrain_utils as tu
from humanoid.utils.terrain import HumanoidTerrain


def _cfg(**kw):
    c = XBotLCfg().terrain
    c.mesh_type = "heightfield"
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def test_layout_and_determinism():
    np.random.seed(5)
    a = HumanoidTerrain(_cfg(), 4096)
    np.random.seed(5)
    b = HumanoidTerrain(_cfg(), 4096)
    assert a.heightsamples.shape == (2100, 2100) and a.heightsamples.dtype == np.int16
    np.testing.assert_array_equal(a.heightsamples, b.heightsamples)
    border = a.border
    assert border == 250
    assert not a.heightsamples[:border].any() and not a.heightsamples[-border:].any()
    assert not a.heightsamples[:, :border].any() and not a.heightsamples[:, -border:].any()
    # obstacles <= 0.04 m, random uniform <= 0.07 m, slopes 0.15 * 4 m, stairs 0.04 m / 0.4 m tread
    assert np.abs(a.heightsamples).max() * 0.005 < 0.65
    # origin z = max height of the central 2 x 2 m of each sub-terrain
    for i, j in [(0, 0), (7, 13), (19, 19)]:
        sub = a.heightsamples[250 + 80 * i:250 + 80 * (i + 1), 250 + 80 * j:250 + 80 * (j + 1)]
        np.testing.assert_allclose(a.env_origins[i, j], [(i + 0.5) * 8, (j + 0.5) * 8, sub[30:50, 30:50].max() * 0.005])


def test_mix_follows_proportions():
    np.random.seed(0)
    t = HumanoidTerrain(_cfg(num_rows=40, num_cols=40), 1)
    subs = t.heightsamples[t.border:-t.border, t.border:-t.border].reshape(40, 80, 40, 80).transpose(0, 2, 1, 3)
    flat = np.mean([not s.any() for s in subs.reshape(-1, 80, 80)])
    assert 0.12 < flat < 0.30  # proportion 0.2 (+ near-zero difficulty draws)


def _sub(n=80):
    return tu.SubTerrain(width=n, length=n, vertical_scale=0.005, horizontal_scale=0.1)


def test_pyramid_sloped_symmetric_and_clipped():
    t = tu.pyramid_sloped_terrain(_sub(), slope=0.15, platform_size=1.0)
    h = t.height_field_raw
    assert np.abs(h.astype(int) - h.T).max() <= 1  # float products truncated to int16
    assert h.min() == 0 and h[40, 40] == h.max()
    assert (h[37:43, 37:43] == h.max()).all()  # clipped platform


def test_stairs_monotone_to_platform():
    t = tu.pyramid_stairs_terrain(_sub(), step_width=0.4, step_height=0.04, platform_size=1.0)
    row = t.height_field_raw[40, :40]
    assert (np.diff(row) >= 0).all() and row[0] == 0 and row[-1] == row.max()
    assert set(np.unique(row)) <= set(range(0, 200, 8))


def test_random_uniform_bounds():
    np.random.seed(1)
    t = tu.random_uniform_terrain(_sub(), min_height=-0.07, max_height=0.07, step=0.005, downsampled_scale=0.2)
    h = t.height_field_raw
    assert h.min() >= -14 and h.max() <= 14 and h.std() > 2


def test_discrete_obstacles_platform():
    np.random.seed(2)
    t = tu.discrete_obstacles_terrain(_sub(), 0.04, 1.0, 2.0, 20, platform_size=3.0)
    h = t.height_field_raw
    assert set(np.unique(h)) <= {-8, -4, 0, 4, 8}
    assert not h[25:55, 25:55].any()


def test_trimesh_shapes():
    hf = np.random.RandomState(0).randint(-5, 5, size=(6, 7)).astype(np.int16)
    v, tri = tu.convert_heightfield_to_trimesh(hf, 0.1, 0.005, 0.75)
    assert v.shape == (42, 3) and tri.shape == (2 * 5 * 6, 3) and tri.max() < 42
    np.testing.assert_allclose(v[:, 2], hf.flatten() * 0.005, rtol=1e-6)
