"""Native risk_accumulate list pass == the reference's Python semantics, bit for bit
(ref ops/risk_accumulate.py:10-77; SURVEY Appendix A goldens)."""
import random

import pytest

from ops.risk_accumulate import risk_accumulate


def _both(monkeypatch, payload):
    monkeypatch.setenv("RISK_DEVICE", "cpu")
    monkeypatch.setenv("RISK_NATIVE", "0")
    try:
        ref = risk_accumulate(payload)
    except Exception as exc:  # noqa: BLE001
        ref = (type(exc), str(exc))
    monkeypatch.setenv("RISK_NATIVE", "1")
    try:
        got = risk_accumulate(payload)
    except Exception as exc:  # noqa: BLE001
        got = (type(exc), str(exc))
    if isinstance(ref, dict):
        ref.pop("compute_time_ms")
        got.pop("compute_time_ms")
    return ref, got


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_values_bit_identical(monkeypatch, seed):
    rng = random.Random(seed)
    vals = []
    for _ in range(20000):
        r = rng.random()
        if r < 0.5:
            vals.append(rng.uniform(-1e6, 1e6))
        elif r < 0.7:
            vals.append(rng.randint(-10**12, 10**12))
        elif r < 0.85:
            vals.append(f"  {rng.uniform(-5, 5)!r} ")
        elif r < 0.9:
            vals.append(rng.choice([True, False]))
        else:
            vals.append(rng.choice(["1e3", "-0.0", "1_000", 3.0e-320, -0.0]))
    ref, got = _both(monkeypatch, {"values": vals})
    assert got == ref
    ref, got = _both(monkeypatch, {"values": vals + ["inf", 1.0, "-inf"]})  # nan sum: compare reprs
    assert repr(got) == repr(ref)


def test_items_and_errors(monkeypatch):
    items = [{"risk": 1}, {"x": 2}, {"risk": "4"}, {"risk": True}, {"p": 3, "risk": 2.5}]
    assert _both(monkeypatch, {"items": items}) == _both(monkeypatch, {"items": items})[::-1]
    ref, got = _both(monkeypatch, {"items": [{"p": 1}, {"p": 3}], "field": "p"})
    assert got == ref == {"count": 2, "sum": 4.0, "mean": 2.0, "min": 1.0, "max": 3.0}
    for bad in ({"values": [None]}, {"values": [1, "x"]}, {"values": [[1]]}, {"items": [1]},
                {"items": [{"risk": None}]}, {"values": [10**400]}, {"values": "x"}, {}):
        ref, got = _both(monkeypatch, bad)
        assert got == ref and isinstance(ref, tuple), (bad, ref, got)
    ref, got = _both(monkeypatch, {"values": []})
    assert got == ref == {"count": 0, "sum": 0.0, "mean": 0.0, "min": None, "max": None}
