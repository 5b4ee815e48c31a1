"""GAE oracle against golden vectors from the reference RolloutStorage.compute_returns."""
import numpy as np
import pytest

import envlogic_ref as E


@pytest.mark.parametrize("N", [4, 64])
def test_gae_oracle(golden, N):
    g = golden("gae.npz")
    ret, adv = E.gae(g[f"N{N}_rewards"], g[f"N{N}_dones"], g[f"N{N}_values"], g[f"N{N}_last_values"], 0.994, 0.9)
    np.testing.assert_array_equal(ret, g[f"N{N}_returns"])   # same fp32 op order -> bitwise
    np.testing.assert_allclose(adv, g[f"N{N}_advantages"], rtol=1e-5, atol=1e-6)
