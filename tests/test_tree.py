"""Host tree bookkeeping (tree.py) — level structure as the reference builds it
(SURVEY.md §8(a) sizes, src/m_build_tree.f90:51-72) and load balance."""
import numpy as np
import pytest

from tests.mgdriver import omg

T = omg.tree


def rect(domain, box, smoother=T.MG_SMOOTHER_GSRB, periodic=False, n_cpu=1):
    t = T.MGTree()
    t.smoother_type = smoother
    t.n_cpu = n_cpu
    d = np.array(domain)
    t.build_rectangle(d, box, 1.0 / d, [0, 0, 0], [periodic] * 3, 0)
    t.load_balance()
    return t


@pytest.mark.parametrize("domain,box,levels,first", [
    ((64, 64, 64), 8, (-4, 1), -2),
    ((256, 256, 256), 16, (-6, 1), -3),
    ((512, 512, 512), 16, (-7, 1), -4),
])
def test_level_structure(domain, box, levels, first):
    t = rect(domain, box)
    assert (t.lowest_lvl, t.highest_lvl) == levels
    assert t.first_normal_lvl == first
    n1 = np.prod(np.array(domain) // box)
    assert len(t.lvls[1].ids) == n1
    assert len(t.lvls[t.lowest_lvl].ids) == 1
    assert t.box_size_lvl[t.lowest_lvl] == 2


def test_neighbors_symmetric_periodic():
    t = rect((64, 64, 64), 8, periodic=True)
    rev = [2, 1, 4, 3, 6, 5]
    for lvl in range(t.lowest_lvl, 2):
        for id_ in t.lvls[lvl].ids:
            for nb in range(6):
                n = t.neighbors[id_, nb]
                assert n > 0
                assert t.neighbors[n, rev[nb] - 1] == id_


def test_load_balance_morton_chunks():
    t = rect((128, 128, 128), 16, n_cpu=8)
    ranks = t.rank[t.lvls[1].ids]
    assert np.all(np.diff(ranks) >= 0)            # contiguous chunks in id order
    assert np.bincount(ranks).tolist() == [64] * 8
    # levels below first_normal_lvl live on one rank (m_load_balance.f90:81,125-130)
    single = max(t.first_normal_lvl - 1, t.lowest_lvl)
    for lvl in range(t.lowest_lvl, single + 1):
        assert len(set(t.rank[t.lvls[lvl].ids].tolist())) == 1
