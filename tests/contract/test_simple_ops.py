"""Golden I/O of echo / map_tokenize / risk_accumulate."""
import math
import random

import pytest

from ops.echo import echo
from ops.map_tokenize import map_tokenize
from ops.risk_accumulate import risk_accumulate


def test_echo_goldens():
    assert echo(None) == {"ok": True, "echo": {}}
    assert echo([1]) == {"ok": True, "echo": [1], "note": "payload_was_not_dict"}
    assert echo({"a": 1}) == {"ok": True, "echo": {"a": 1}}


@pytest.mark.parametrize("payload,expected", [
    ({"text": "abcdefghij", "chunk_size": 4}, {"ok": True, "tokens": ["abcd", "efgh", "ij"], "count": 3, "total_chars": 10}),
    ({"data": "xyz"}, {"ok": True, "tokens": ["xyz"], "count": 1, "total_chars": 3}),
    ({"items": ["abcde", None, 7], "chunk_size": 2},
     {"ok": True, "tokens": ["ab", "cd", "e", "7"], "count": 4, "total_chars": 6, "items_count": 3}),
    ({"text": "a", "chunk_size": 0}, {"ok": False, "error": "payload.chunk_size must be a positive integer"}),
    ({"text": "a", "chunk_size": 2.0}, {"ok": False, "error": "payload.chunk_size must be a positive integer"}),
    (None, {"ok": True, "tokens": [], "count": 0, "total_chars": 0}),
    ({"text": 123}, {"ok": False, "error": "payload.text must be a string"}),
    ({"items": "abc"}, {"ok": False, "error": "payload.items must be a list of strings"}),
])
def test_map_tokenize_goldens(payload, expected):
    assert map_tokenize(payload) == expected


def _strip(d):
    d = dict(d)
    assert isinstance(d.pop("compute_time_ms"), float)
    return d


def test_risk_goldens():
    assert _strip(risk_accumulate({"values": [1, "2.5", 3]})) == {
        "count": 3, "sum": 6.5, "mean": 2.1666666666666665, "min": 1.0, "max": 3.0}
    assert _strip(risk_accumulate({"items": [{"risk": 1}, {"x": 2}, {"risk": "4"}]})) == {
        "count": 2, "sum": 5.0, "mean": 2.5, "min": 1.0, "max": 4.0}
    assert _strip(risk_accumulate({"items": [{"p": 1}, {"p": 3}], "field": "p"})) == {
        "count": 2, "sum": 4.0, "mean": 2.0, "min": 1.0, "max": 3.0}
    assert _strip(risk_accumulate({"values": []})) == {"count": 0, "sum": 0.0, "mean": 0.0, "min": None, "max": None}
    assert _strip(risk_accumulate({"values": [True]}))["sum"] == 1.0


@pytest.mark.parametrize("payload,msg", [
    ({}, "payload must include either 'values' or 'items'"),
    ({"values": "x"}, "payload.values must be a list"),
    ({"values": [None]}, "value must be numeric"),
    ({"items": [1]}, "payload.items must contain dict objects"),
])
def test_risk_raises(payload, msg):
    with pytest.raises(ValueError, match=msg):
        risk_accumulate(payload)


def test_risk_matches_python_sum_bitwise():
    rng = random.Random(5)
    vals = [rng.uniform(-1e6, 1e6) for _ in range(10000)]
    out = risk_accumulate({"values": vals})
    assert out["sum"] == sum(vals) and out["min"] == min(vals) and out["max"] == max(vals)
    assert math.isclose(out["mean"], sum(vals) / len(vals))
