"""Pins the C++ restatement of the predicates (CPU baseline) to the Python
oracle and the Appendix A.4 table."""
import numpy as np

from oracle import cpu_ref
from tests.golden.kat_cases import cases
from tests.parity import expected_flags, oracle_batch
from tests.workload import make_pairs


def _check(pairs, threads=1):
    d = cpu_ref.DecodedPairs(pairs)
    flags, sweeps, sec = d.decide(threads)
    exp = np.array([expected_flags(r) for r in oracle_batch(pairs)], dtype=np.uint8)
    assert (flags == exp).all(), np.nonzero(flags != exp)[0][:10]
    d.close()


def test_kat():
    _check([(a, b) for _, a, b, _, _ in cases()])


def test_population_threads():
    pairs, _, _ = make_pairs(1500, seed=11, mutate_frac=0.2)
    _check(pairs, threads=4)
