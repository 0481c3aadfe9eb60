"""Pin the CPU oracle against the reference's own run outputs.

The reference ships no tests or golden vectors, and it cannot be built in this
image (DESIGN.md "Oracle").  What pins the restatement are the outputs of the
reference itself recorded in SURVEY.md §8 / §4 (probe runs of the reference
build, copied into tests/golden/known_answers.json): level sizes, active block
counts and CSR sizes per configuration.  These are integer results of the
Morton sort + aggregation and must match exactly.
"""
import json
import os

import numpy as np
import pytest

from conftest import cloth, tet

KA = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "known_answers.json")))


def _oracle(mesh, L):
    from oracle import Oracle
    o = Oracle(mesh.nV, 0, 0, L, 1)
    o.allocate(mesh)
    o.prepare(mesh)
    return o


@pytest.mark.parametrize("name", ["10k", "256k", "1M"])
def test_cloth_level_sizes(name):
    ka = KA["configs"][name]
    mesh = cloth(ka["W"])
    assert mesh.nnz == ka["nnz"]
    o = _oracle(mesh, ka["levels"])
    assert o.natural_levels == ka["natural_levels"]
    ls = o.level_size()
    sizes = [mesh.nV] + [int(x) for x in ls[1: ka["levels"], 0]]
    assert sizes == ka["level_sizes"][: ka["levels"]]
    assert o.total_clusters // 32 == ka["active_blocks"]
    assert o.capacity == ka["capacity"]


@pytest.mark.slow
def test_tet_4m_level_sizes():
    ka = KA["configs"]["4M-tet"]
    mesh = tet(ka["W"])
    assert mesh.nnz == ka["nnz"]
    o = _oracle(mesh, ka["levels"])
    ls = o.level_size()
    sizes = [mesh.nV] + [int(x) for x in ls[1: ka["levels"], 0]]
    assert sizes == ka["level_sizes"]
    assert o.total_clusters // 32 == ka["active_blocks"]


def test_level_count_rule():
    # ComputeLevelNums (.cpp:112-135): natural levels and the 1.5x capacity
    from oracle import Oracle
    for nV, L, cap in [(10_000, 3, 15552), (262_144, 4, 405936), (1_048_576, 4, 1623600), (4_096_000, 5, 6342240)]:
        o = Oracle(nV, 0, 0, 0, 1)
        assert (o.natural_levels, o.capacity) == (L, cap)


def test_more_than_five_levels_rejected():
    from oracle import Oracle
    with pytest.raises(ValueError):
        Oracle(40_000_000, 0, 0, 0, 1)   # natural L = 6 (B-6)
