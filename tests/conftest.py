"""Shared test setup: import paths, the `gpu` marker, cached meshes."""
import functools
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "preconditioner-for-cloth-and-deformable-body-simulation_amd")
for p in (os.path.join(PKG, "python"), os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: large configurations (minutes)")


@functools.lru_cache(maxsize=None)
def cloth(W):
    from mas_amd import meshgen
    return meshgen.cloth_grid(W)


@functools.lru_cache(maxsize=None)
def tet(W):
    from mas_amd import meshgen
    return meshgen.tet_lattice(W)


@pytest.fixture(scope="session")
def meshes():
    return {"cloth": cloth, "tet": tet}
