"""CPU tests of two oracle helpers the GPU contact / config-4 tests rely on.

  * physics_ref.ground: the numpy restatement of physics_ref.c's `ground` (the triangulated
    heightfield under a point) — heights at the samples, the (i, j)-(i+1, j+1) split (every
    point on the plane of its triangle's three vertices), unit upward normals, the plane case;
  * pipeline_ref.PhiloxDraws with a shard offset: the draws of envs [off, off + n) of an
    N-env job equal rows [off, off + n) of the whole job's draws (the kernels key every stream by
    the global env id).
"""
import numpy as np

import physics_ref as P
import pipeline_ref as PR


class _HfCfg:
    terrain_type = 1
    hf_horizontal_scale = 0.1
    hf_vertical_scale = 0.005
    hf_border = 1.0
    hf_rows = 40
    hf_cols = 30


def test_ground_interpolates_the_triangles():
    c = _HfCfg()
    rng = np.random.default_rng(0)
    hf = rng.integers(-40, 40, size=(c.hf_rows, c.hf_cols)).astype(np.int16)
    i, j = rng.integers(0, c.hf_rows - 1, 500), rng.integers(0, c.hf_cols - 1, 500)
    x, y = i * c.hf_horizontal_scale - c.hf_border, j * c.hf_horizontal_scale - c.hf_border
    h, n = P.ground(c, hf, x, y)
    np.testing.assert_allclose(h, hf[i, j] * c.hf_vertical_scale, atol=1e-12)  # the samples
    np.testing.assert_allclose(np.linalg.norm(n, axis=-1), 1.0, atol=1e-12)
    # every point of a triangle lies on the plane through its three vertices, normal up
    u, v = rng.uniform(0, 1, 500), rng.uniform(0, 1, 500)
    px, py = x + u * c.hf_horizontal_scale, y + v * c.hf_horizontal_scale
    h, n = P.ground(c, hf, px, py)
    H = hf.astype(np.float64) * c.hf_vertical_scale
    lower = u >= v                      # (i,j), (i+1,j), (i+1,j+1) ; else (i,j), (i,j+1), (i+1,j+1)
    vi = np.where(lower, i + 1, i)
    vj = np.where(lower, j, j + 1)
    for ai, aj in ((i, j), (vi, vj), (i + 1, j + 1)):
        vx, vy = ai * c.hf_horizontal_scale - c.hf_border, aj * c.hf_horizontal_scale - c.hf_border
        d = (vx - px) * n[:, 0] + (vy - py) * n[:, 1] + (H[ai, aj] - h) * n[:, 2]
        np.testing.assert_allclose(d, 0.0, atol=1e-12)
    assert (n[:, 2] > 0).all()
    flat = P.ground(type("Plane", (), {"terrain_type": 0})(), None, px, py)
    assert (flat[0] == 0).all() and (flat[1][:, 2] == 1).all()


def test_quat_rotate_matches_rotation_matrix():
    from scipy.spatial.transform import Rotation
    rng = np.random.default_rng(1)
    q = rng.standard_normal((64, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    v = rng.standard_normal((64, 3))
    np.testing.assert_allclose(P.quat_rotate(q, v), Rotation.from_quat(q).apply(v), atol=1e-12)


def test_shard_draws_are_the_whole_jobs_rows():
    N, n, off, seed = 96, 16, 64, 11
    whole, shard = PR.PhiloxDraws(seed, N), PR.PhiloxDraws(seed, n, off)
    sl = slice(off, off + n)
    np.testing.assert_array_equal(shard.act_delay(5), whole.act_delay(5)[sl])
    np.testing.assert_array_equal(shard.act_noise(5, 12), whole.act_noise(5, 12)[sl])
    np.testing.assert_array_equal(shard.obs_noise(7, 47), whole.obs_noise(7, 47)[sl])
    for a, b in zip(shard.push(400), whole.push(400)):
        np.testing.assert_array_equal(a, b[sl])
    rid = np.array([0, 3, 9])
    np.testing.assert_array_equal(shard.reset_dof(rid, 9, 12), whole.reset_dof(rid + off, 9, 12))
    np.testing.assert_array_equal(shard.reset_root(rid, 9), whole.reset_root(rid + off, 9))
    np.testing.assert_array_equal(shard.terrain_level(rid, 9, 10), whole.terrain_level(rid + off, 9, 10))
    for a, b in zip(shard.cmd(rid, 9, 1), whole.cmd(rid + off, 9, 1)):
        np.testing.assert_array_equal(a, b)
    # and the shard's own ids are not the first rows of the job
    assert not np.array_equal(shard.act_noise(5, 12), whole.act_noise(5, 12)[:n])
