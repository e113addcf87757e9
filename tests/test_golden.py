"""The float64 oracle reproduces the committed golden vectors (tests/golden/oracle_cases.npz):
pins the oracle, the host-side model construction and the parameter bridge against drift."""
import numpy as np
import pytest

from tests.golden_util import cases, load_case
from tests.parity_util import oracle_reference


@pytest.mark.parametrize("name", cases())
def test_oracle_reproduces_golden(name):
    model, batch, eps, x0, elbo_ref, grad_ref = load_case(name, "cpu")
    elbo, grads = oracle_reference(model, batch, eps, x0)
    assert np.allclose(elbo, elbo_ref, rtol=1e-10, atol=0.0)
    g = np.concatenate([np.asarray(grads[n], dtype=np.float64).ravel() for n in model.store.names()])
    assert np.linalg.norm(g - grad_ref) <= 1e-6 * np.linalg.norm(grad_ref)
