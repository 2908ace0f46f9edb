"""Multi-rank parity on one GPU: the golden runs the reference made at 2, 4
and 8 MPI ranks (tests/golden/golden.json), replayed by as many device
contexts exchanging through the loopback transport (include/omg.h,
omg_loopback_unique_id).  Same tree partition (mg_load_balance), same halo /
restriction / prolongation plans and kernels as the RCCL path; the periodic
cases pin the MPICH pairwise order of the get_sum allreduce per rank count."""
import json
import os

import pytest

from tests.mgdriver import run_problem_loopback

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))["configs"]
MULTI = [(n, int(r)) for n, e in sorted(GOLDEN.items()) for r in e["runs"] if int(r) > 1]

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,ranks", MULTI)
def test_multirank_matches_reference_golden(name, ranks):
    e = GOLDEN[name]
    out = run_problem_loopback(e["args"], ranks)
    assert out["history"] == e["runs"][str(ranks)]["history"]


# Replicated coarse levels (omg_set_coarse_replication): every coarse level
# on every rank (1 << 40 cells), or only the smallest ones (4096 cells, so the
# restriction into a replicated level from a distributed one is exercised at
# several box sizes).  Same bits as the reference's distributed coarse levels.
@pytest.mark.parametrize("rep", [1 << 40, 4096])
@pytest.mark.parametrize("name,ranks", MULTI)
def test_multirank_replicated_coarse_matches_golden(name, ranks, rep):
    e = GOLDEN[name]
    out = run_problem_loopback(e["args"], ranks, rep_cells=rep)
    assert out["history"] == e["runs"][str(ranks)]["history"]
