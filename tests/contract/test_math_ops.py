"""CPU ops restored from the reference's OP_TO_MODULE map:
fibonacci, prime_factor, sat_verify, subset_sum — goldens and brute force
(parity unpinned: the reference never shipped these modules)."""
import itertools
import random

import pytest

from ops.fibonacci import fibonacci
from ops.prime_factor import prime_factor
from ops.sat_verify import sat_verify
from ops.subset_sum import subset_sum


def test_fibonacci():
    assert fibonacci({"n": 0}) == {"ok": True, "n": 0, "value": 0, "digits": 1}
    assert fibonacci({"n": 10})["value"] == 55
    assert fibonacci({"n": 78})["value"] == 8944394323791464  # < 2**53
    big = fibonacci({"n": 100})
    assert big["value"] == "354224848179261915075" and big["digits"] == 21
    assert fibonacci({"n": 5, "count": 4})["sequence"] == [5, 8, 13, 21]
    assert fibonacci({"n": 1000})["digits"] == 209
    for bad in ({"n": -1}, {"n": 1.0}, {"n": True}, {}, {"n": 2_000_000}, {"n": 3, "count": 0}):
        assert fibonacci(bad)["ok"] is False
    assert fibonacci([1]) == {"ok": False, "error": "payload must be a dict"}


def test_prime_factor():
    assert prime_factor({"n": 1}) == {"ok": True, "n": 1, "factors": [], "is_prime": False}
    assert prime_factor({"n": 97})["is_prime"] is True
    assert prime_factor({"n": 561})["factors"] == [3, 11, 17]  # Carmichael
    assert prime_factor({"n": 2 ** 10 * 3 ** 4})["factors"] == [2] * 10 + [3] * 4
    p, q = 4294967291, 4294967279  # two 32-bit primes
    assert prime_factor({"n": p * q})["factors"] == [q, p]
    r = prime_factor({"n": str((2 ** 61 - 1) * 1000003)})
    assert r["factors"] == [1000003, str(2 ** 61 - 1)] and r["n"] == str((2 ** 61 - 1) * 1000003)
    rng = random.Random(0)
    for _ in range(200):
        n = rng.randrange(2, 10 ** 6)
        f = prime_factor({"n": n})["factors"]
        prod = 1
        for x in f:
            prod *= x
        assert prod == n and f == sorted(f)
    for bad in ({"n": 0}, {"n": -5}, {"n": 2 ** 97}, {"n": "12a"}):
        assert prime_factor(bad)["ok"] is False


def test_sat_verify():
    cnf = [[1, -2], [2, 3], [-1, -3]]
    assert sat_verify({"cnf": cnf, "assignment": {"1": True, "2": True, "3": False}})["satisfied"] is True
    assert sat_verify({"cnf": cnf, "assignment": [True, True, False]})["satisfied"] is True
    r = sat_verify({"cnf": cnf, "assignment": [1, 2, 3]})
    assert r["satisfied"] is False and r["unsatisfied_clauses"] == [2] and r["clauses"] == 3
    assert sat_verify({"cnf": [[1]], "assignment": {}})["satisfied"] is False  # unassigned = false
    assert sat_verify({"cnf": [[0]], "assignment": []})["ok"] is False
    assert sat_verify({"cnf": "x", "assignment": []})["ok"] is False


def _brute(values, target):
    for k in range(len(values) + 1):
        for c in itertools.combinations(range(len(values)), k):
            if sum(values[i] for i in c) == target:
                return True
    return False


def test_subset_sum_brute_force():
    rng = random.Random(1)
    for _ in range(300):
        n = rng.randrange(0, 11)
        values = [rng.randrange(-20, 40) for _ in range(n)]
        target = rng.randrange(-30, 80)
        r = subset_sum({"values": values, "target": target})
        assert r["ok"] and r["found"] == _brute(values, target), (values, target)
        if r["found"]:
            assert sum(values[i] for i in r["indices"]) == target
            assert r["subset"] == [values[i] for i in r["indices"]]
            assert r["indices"] == sorted(set(r["indices"]))


def test_subset_sum_meet_in_middle():
    rng = random.Random(2)
    values = [rng.randrange(1, 2 ** 40) for _ in range(30)]
    pick = rng.sample(range(30), 9)
    target = sum(values[i] for i in pick)
    r = subset_sum({"values": values, "target": target})
    assert r["found"] and r["method"] == "meet_in_the_middle" and sum(values[i] for i in r["indices"]) == target
    assert subset_sum({"values": [2 ** 40, 3 * 2 ** 40], "target": 7})["found"] is False
    assert subset_sum({"values": [2 ** 40 + i for i in range(60)], "target": 1})["ok"] is False
    assert subset_sum({"values": [1, 2.5], "target": 3})["ok"] is False
